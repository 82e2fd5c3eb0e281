// MI355X (gfx950) kernels for Kopia's content-defined-chunking splitters.
//
// Reference semantics (bit-exact):
//   buzhash32Splitter.NextSplitPoint   repo/splitter/splitter_buzhash32.go:26-67
//   rabinKarp64Splitter.NextSplitPoint repo/splitter/splitter_rabinkarp64.go:26-67
//   fixedSplitter.NextSplitPoint       repo/splitter/splitter_fixed.go:15-26
//
// Key identity: the rolling hash is never reset inside a
// stream and always equals the hash of the 64 bytes ending at the current
// position (zero bytes before the stream start).  So cand(p) := hash(p) & mask
// == 0 is a pure function of bytes p-63..p, and the chunk rule is: from chunk
// start s, cut after the first p in [s+min-1, s+max-1] with cand(p), else after
// s+max-1.  The reference's fast path (only the last 64 of the first min-1
// bytes are rolled) becomes "start scanning at s+min-64": bytes before that are
// never read.
//
// Kernels:
//   split_batch_pipe_kernel  the batch hot path (buzhash): persistent waves, one stream per
//       wave at a time through a ticketed ring queue; a stream is walked in TILES of 64
//       lanes x L bytes of its test region [s+min-1, s+max-1], lane l hashing segment l
//       after warming up on the 64 bytes before it.  Bytes arrive by LDS-DMA in 128-byte
//       steps; per byte one v_perm (table address), one ds_read of the 64x replicated
//       table (lane l hits bank l%32), a T-ring register for the leaving byte, v_alignbit
//       and v_bitop3, and a running v_min3 candidate test in the rotated frame.  A step
//       whose min passes is re-run exactly; the earliest lane's candidate is the cut.
//   split_batch_rk_kernel    the Rabin-Karp batch walk (two chains per lane).
//   cand_scan_dma_kernel / cand_scan_rk_kernel, seg_prefix, compact, resolve   the long path.
//   scan_first_kernel        one region's first candidate (streaming handle).
//   split_fixed_kernel       FIXED names (reads no data).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <mutex>
#include <type_traits>
#include <vector>
#include <string>

#include "kcdc_internal.h"

namespace kcdc {
namespace dev {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;
constexpr int kBlk = 128;               // bytes per lane per step (one cache line)
constexpr int kNdw = kBlk / 4;          // dwords per lane per step
constexpr int64_t kLaneMax = 2048;      // max bytes per lane segment (tile = 64 x kLaneMax)
#ifndef KCDC_TILE_DIV
#define KCDC_TILE_DIV 256
#endif
constexpr uint64_t kTileDiv = KCDC_TILE_DIV;  // batch lane segments <= avg / kTileDiv (tiles ~ avg / 4), >= 256 B
#ifndef KCDC_BUZ_LANE_MAX
#define KCDC_BUZ_LANE_MAX 2048
#endif
constexpr uint64_t kBuzLaneMax = KCDC_BUZ_LANE_MAX;  // the buzhash batch kernel's lane segment cap
constexpr int kSchedWindow = 16;        // bytes per scheduling window in the warm-up / exact loops
constexpr int kLookahead = 16;          // 128-byte steps: table reads issued this many bytes ahead (VGPR bound)

enum Mode { kWarm = 0, kFast = 1 };

__device__ __forceinline__ uint32_t rotl1(uint32_t h) { return __builtin_amdgcn_alignbit(h, h, 31); }
__device__ __forceinline__ uint32_t rotl_n(uint32_t v, uint32_t r) { return r ? (v << r) | (v >> (32 - r)) : v; }

// h' = rotl(h,1) ^ a ^ b as ONE v_bitop3 (truth table 0x96 = 3-input XOR; gfx950 has no
// v_xor3).  hipcc otherwise emits xor + bitop3 per byte.  The builtin, not inline asm:
// the hazard recognizer pads inline-asm VALU with s_nops (76 per 128 bytes).
__device__ __forceinline__ uint32_t roll3(uint32_t h, uint32_t a, uint32_t b) {
    return __builtin_amdgcn_bitop3_b32(rotl1(h), a, b, 0x96);
}

__device__ __forceinline__ uint64_t uni64(uint64_t x) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(x));
    const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(x >> 32));
    return (static_cast<uint64_t>(hi) << 32) | lo;
}

// Byte i of a block held as dwords.
template <int N>
__device__ __forceinline__ uint32_t byte_at(const uint32_t (&dw)[N], int i) {
    return __builtin_amdgcn_perm(0u, dw[i >> 2], 0x0c0c0c00u | static_cast<uint32_t>(i & 3));
}

// ---------------------------------------------------------------- loaders
// A stream is addressed in "coordinates" c = position + off0 relative to the
// 16-byte-aligned base `abase`; coordinates < off0 are the virtual zero bytes
// before the stream start.  Loads go through a buffer descriptor whose range
// check returns zeros for out-of-range (including negative) offsets.
struct Loader {
    __amdgpu_buffer_rsrc_t rsrc;
    u32x4 d;       // the same descriptor as four dwords (operand of the inline-asm LDS-DMA)
    int64_t tb;    // coordinate of descriptor offset 0
    int64_t off0;  // stream misalignment (0..15)

    template <int N>
    __device__ __forceinline__ void load(int64_t c, uint32_t (&dw)[N]) const {
        const int32_t vo = static_cast<int32_t>(c - tb);
#pragma unroll
        for (int j = 0; j < N / 4; j++) {
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, vo + 16 * j, 0, 0);
            dw[4 * j + 0] = v.x;
            dw[4 * j + 1] = v.y;
            dw[4 * j + 2] = v.z;
            dw[4 * j + 3] = v.w;
        }
        if (c == 0 && off0) {  // zero the bytes that precede the stream in its first granule
#pragma unroll
            for (int d = 0; d < 4; d++) {
                const int64_t keep_from = off0 - 4 * d;  // first byte of dword d to keep
                const uint32_t m = keep_from <= 0 ? 0xFFFFFFFFu
                                                  : (keep_from >= 4 ? 0u : (0xFFFFFFFFu << (8 * keep_from)));
                dw[d] &= m;
            }
        }
    }
};

__device__ __forceinline__ Loader make_loader(const uint8_t* abase, int64_t off0, int64_t nbytes_coord, int64_t tb) {
    // tb >= 0 and a multiple of 16; the descriptor covers [tb, round_up16(nbytes_coord)).
    int64_t nrec = ((nbytes_coord + 15) & ~int64_t(15)) - tb;
    if (nrec > 0x7FFFFF00ll) nrec = 0x7FFFFF00ll;
    if (nrec < 0) nrec = 0;
    Loader L;
    L.rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(abase + tb), static_cast<short>(0),
                                               static_cast<int>(nrec), 0x00020000);
    const uint64_t base = reinterpret_cast<uint64_t>(abase + tb);
    L.d.x = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(base));
    L.d.y = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(base >> 32) & 0xFFFFu);  // stride 0
    L.d.z = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(nrec));
    L.d.w = 0x00020000u;
    L.tb = tb;
    L.off0 = off0;
    return L;
}

// ------------------------------------------------------------------ hashes
// Both hashes keep `prev`: the 64 bytes before the current step (the bytes that
// leave the window while the step's bytes enter it).  block<MODE, N>(dw) rolls
// the 4N bytes of dw; byte i leaves-byte is (prev ++ dw)[i].

// buzhash32: h(p) = rotl(h(p-1),1) ^ T[b[p-64]] ^ T[b[p]]  (rollinghash Roll with
// window 64: rotl(T[leave], 64 % 32 = 0)).
struct BuzShared {
    __attribute__((aligned(16))) uint32_t tab[256 * 64];  // tab[v*64 + r] = T[v]  (64 KiB, replica r read by lane r)
};
// Fill the replicated table at kernel start: one global load per thread (two threads per
// entry, 32 replicas each, as four-dword stores rotated by entry so a store instruction's
// lanes spread over the banks).  The loop of one load per replica took 4 dependent rounds of
// L2 loads at every workgroup's start.
__device__ __forceinline__ void fill_buz_table(BuzShared& sm, const uint32_t* buz, uint32_t rot) {
    static_assert(sizeof(BuzShared) == 256 * 64 * 4, "table layout");
    for (uint32_t t = threadIdx.x; t < 512u; t += blockDim.x) {
        const uint32_t e = t & 255u, h = t >> 8;
        const uint32_t v = rotl_n(buz[e], rot);
        const u32x4 q = {v, v, v, v};
        u32x4* row = reinterpret_cast<u32x4*>(sm.tab + e * 64u + h * 32u);
#pragma unroll
        for (uint32_t k = 0; k < 8; k++) row[(k + e) & 7u] = q;
    }
}

// buzhash32 with a register T-ring: ring[j] holds T[b] of the j-th of the 64 bytes
// before the current step, so each byte costs ONE table read (the entering byte);
// the leaving byte's value comes from the ring (first half of a 128-byte step) or
// from the step's own first half (second half), and the second half refills the
// ring in place.  No register rotation at the step boundary: ring[j] dies at byte
// j and is reborn at byte 64+j.
struct BuzRing {
    const char* tab;
    uint32_t lane4;
    uint32_t mask;
    uint32_t h;
    uint32_t ring[64];
    using State = uint32_t;
    __device__ __forceinline__ State save() const { return h; }
    __device__ __forceinline__ uint32_t look(uint32_t dwv, int k) const {
        const uint32_t a = __builtin_amdgcn_perm(dwv, lane4, 0x0c0c0000u | ((4u + k) << 8));
        return *reinterpret_cast<const uint32_t*>(tab + a);
    }
    __device__ __forceinline__ void clear() {
        h = 0;
#pragma unroll
        for (int i = 0; i < 64; i++) ring[i] = 0;
    }
    template <int MODE, int N>
    __device__ __forceinline__ uint32_t block(const uint32_t (&dw)[N]) {
        static_assert(N == 16 || N == 32, "T-ring steps are 64 or 128 bytes");
        uint32_t m = 0xFFFFFFFFu;
        if constexpr (MODE == kWarm) {  // 64 bytes on a zero history: G-recurrence warm-up
#pragma unroll
            for (int i = 0; i < 64; i++) {
                if (kSchedWindow && i % kSchedWindow == 0) __builtin_amdgcn_sched_barrier(0);
                const uint32_t t = look(dw[i >> 2], i & 3);
                h = rotl1(h) ^ t;
                ring[i] = t;
            }
            return m;
        } else if constexpr (N == 16) {
#pragma unroll
            for (int i = 0; i < 64; i++) {
                if (kSchedWindow && i % kSchedWindow == 0) __builtin_amdgcn_sched_barrier(0);
                const uint32_t t = look(dw[i >> 2], i & 3);
                h = roll3(h, ring[i], t);
                ring[i] = t;
                m = min(m, h & mask);
                if ((i & 3) == 3) asm volatile("" : "+v"(m));
            }
            return m;
        } else {
            uint32_t loc[64];
#pragma unroll
            for (int i = 0; i < 64; i++) {
                if (kSchedWindow && i % kSchedWindow == 0) __builtin_amdgcn_sched_barrier(0);
                const uint32_t t = look(dw[i >> 2], i & 3);
                h = roll3(h, ring[i], t);
                loc[i] = t;
                m = min(m, h & mask);
                if ((i & 3) == 3) asm volatile("" : "+v"(m));
            }
#pragma unroll
            for (int i = 64; i < 128; i++) {
                if (kSchedWindow && i % kSchedWindow == 0) __builtin_amdgcn_sched_barrier(0);
                const uint32_t t = look(dw[i >> 2], i & 3);
                h = roll3(h, loc[i - 64], t);
                ring[i - 64] = t;
                m = min(m, h & mask);
                if ((i & 3) == 3) asm volatile("" : "+v"(m));
            }
            return m;
        }
    }
    // A whole 128-byte step (the 128-byte-run DMA path): bytes 0..63 consume the ring and
    // fill loc, bytes 64..127 consume loc and refill the ring (loc[b] can take ring[b]'s
    // register).  Table reads run one 16-byte window ahead of the arithmetic.
    // Positions 0..62 keep their own running min m0, or-ed with hmask at the end.
    template <bool TOP>
    __device__ __forceinline__ uint32_t step128(const uint32_t (&dw)[32], uint32_t hmask) {
        constexpr int W = kLookahead;  // bytes per lookahead window
        uint32_t loc[64];
        uint32_t m = 0xFFFFFFFFu, m0 = 0xFFFFFFFFu;
        uint32_t tw[W], tn[W];
#pragma unroll
        for (int i = 0; i < W; i++) tw[i] = look(dw[i >> 2], i & 3);
#pragma unroll
        for (int w = 0; w < 128 / W; w++) {
            __builtin_amdgcn_sched_barrier(0);
            if (w < 128 / W - 1) {
#pragma unroll
                for (int i = 0; i < W; i++) tn[i] = look(dw[(W * (w + 1) + i) >> 2], i & 3);
            }
#pragma unroll
            for (int i = 0; i < W; i++) {
                const int b = W * w + i;
                if (b < 64) {
                    h = roll3(h, ring[b], tw[i]);
                    loc[b] = tw[i];
                } else {
                    h = roll3(h, loc[b - 64], tw[i]);
                    ring[b - 64] = tw[i];
                }
                const uint32_t t = TOP ? h : h & mask;
                if (b < 63) {
                    m0 = min(m0, t);
                    if ((b & 3) == 3) asm volatile("" : "+v"(m0));
                } else {
                    m = min(m, t);
                    if ((b & 3) == 3) asm volatile("" : "+v"(m));
                }
            }
#pragma unroll
            for (int i = 0; i < W; i++) tw[i] = tn[i];
        }
        return min(m, m0 | hmask);
    }
    // The rare exact re-run of a step whose running test passed: the first position in [lo, hi]
    // that is a candidate, else 4N.  16-byte windows (the arrays shift by four dwords per window),
    // done as soon as every lane running it has found its candidate.  (Round 5: the arrays shifted
    // by one dword every 4 bytes, ~3,800 VALU per re-run, and at 128K averages 6 % of wave-steps
    // re-run.  Fully unrolled instead, the long-path scan kernel spilled.)
    template <int N>
    __device__ __forceinline__ uint32_t exact(State st0, const uint32_t (&prv)[16], const uint32_t (&dw)[N], int lo,
                                              int hi) const {
        static_assert(N % 4 == 0, "16-byte windows");
        uint32_t e[N], o[N];
#pragma unroll
        for (int j = 0; j < N; j++) {
            e[j] = dw[j];
            o[j] = j < 16 ? prv[j] : dw[j - 16];
        }
        uint32_t hh = st0, first = 4 * N;
#pragma unroll 1
        for (int w = 0; w < N / 4; w++) {
#pragma unroll
            for (int b = 0; b < 16; b++) {
                hh = rotl1(hh) ^ look(o[b >> 2], b & 3) ^ look(e[b >> 2], b & 3);
                const int i = 16 * w + b;
                if (first == 4 * N && (hh & mask) == 0 && i >= lo && i <= hi) first = static_cast<uint32_t>(i);
            }
            if (__ballot(first == 4 * N) == 0) break;
#pragma unroll
            for (int k = 0; k < N - 4; k++) {
                e[k] = e[k + 4];
                o[k] = o[k + 4];
            }
        }
        return first;
    }
};

// rabinkarp64: v ^= out[b[p-64]]; idx = v >> shift; v = (v << 8 | b[p]) ^ mod[idx].
struct RabinShared {
    uint64_t out[256];
    uint64_t mod[256];
};

struct Rabin {
    const RabinShared* tab;
    uint32_t mask;
    uint32_t shift;
    uint64_t v;
    uint32_t prev[16];
    using State = uint64_t;
    __device__ __forceinline__ State save() const { return v; }

    __device__ __forceinline__ void clear() {
        v = 0;
#pragma unroll
        for (int i = 0; i < 16; i++) prev[i] = 0;
    }
    __device__ __forceinline__ uint64_t roll(uint64_t x, uint32_t bo, uint32_t bi) const {
        x ^= tab->out[bo];
        const uint32_t idx = static_cast<uint32_t>(x >> shift) & 0xFFu;
        return ((x << 8) | bi) ^ tab->mod[idx];
    }
    template <int MODE, int N>
    __device__ __forceinline__ uint32_t block(const uint32_t (&dw)[N]) {
        uint32_t m = 0xFFFFFFFFu;
#pragma unroll
        for (int i = 0; i < 4 * N; i++) {
            const uint32_t bo = MODE == kWarm ? 0u : (i < 64 ? byte_at(prev, i) : byte_at(dw, i - 64));
            v = roll(v, bo, byte_at(dw, i));
            if (MODE == kFast) {
                m = min(m, static_cast<uint32_t>(v) & mask);
                if ((i & 3) == 3) asm volatile("" : "+v"(m));
            }
        }
#pragma unroll
        for (int i = 0; i < 16; i++) prev[i] = dw[N - 16 + i];
        return m;
    }
    template <int N>
    __device__ __forceinline__ uint32_t exact(State st0, const uint32_t (&prv)[16], const uint32_t (&dw)[N], int lo,
                                              int hi) const {
        uint32_t e[N], o[N];
#pragma unroll
        for (int j = 0; j < N; j++) {
            e[j] = dw[j];
            o[j] = j < 16 ? prv[j] : dw[j - 16];
        }
        uint64_t vv = st0;
        uint32_t first = 4 * N;
#pragma unroll 1
        for (int j = 0; j < N; j++) {
#pragma unroll
            for (int b = 0; b < 4; b++) {
                vv = roll(vv, (o[0] >> (8 * b)) & 0xFFu, (e[0] >> (8 * b)) & 0xFFu);
                const int i = 4 * j + b;
                if (first == 4 * N && (static_cast<uint32_t>(vv) & mask) == 0 && i >= lo && i <= hi)
                    first = static_cast<uint32_t>(i);
            }
#pragma unroll
            for (int k = 0; k < N - 1; k++) {
                e[k] = e[k + 1];
                o[k] = o[k + 1];
            }
        }
        return first;
    }
};

// --------------------------------------------------------- region scanner
// First candidate coordinate in [lo, hi] (inclusive, lo <= hi), or -1.
// Wave-uniform in and out.  `H` is a prepared hash (tables + mask).
template <class H>
__device__ int64_t scan_region(H hash, const uint8_t* abase, int64_t off0, int64_t nbytes_coord, int64_t lo,
                               int64_t hi, int lane) {
    int64_t ct = lo & ~int64_t(63);
    while (ct <= hi) {
        const int64_t rem = hi - ct + 1;
        int64_t per = (rem + kWave - 1) / kWave;
        per = (per + kBlk - 1) / kBlk * kBlk;
        const int64_t L = per < kLaneMax ? per : kLaneMax;
        const int64_t tb = ct >= 64 ? ct - 64 : 0;
        const Loader ld = make_loader(abase, off0, nbytes_coord, tb);

        const int64_t c0 = ct + lane * L;
        const int nb = static_cast<int>(L / kBlk);
        int64_t found = -1;
        if (c0 <= hi) {
            uint32_t cur[kNdw], nxt[kNdw];
            {
                uint32_t w[16];
                hash.clear();
                ld.load(c0 - 64, w);
                hash.template block<kWarm>(w);  // h = hash of the 64-byte window before c0
            }
            ld.load(c0, cur);
            int k = 0;
            for (;;) {
                bool hit = false;
                typename H::State st0 = hash.save();
                for (; k < nb; k++) {
                    if (c0 + kBlk * k > hi) break;
                    if (k + 1 < nb) ld.load(c0 + kBlk * (k + 1), nxt);
                    st0 = hash.save();
                    if (hash.template block<kFast>(cur) == 0) {
                        hit = true;
                        break;
                    }
#pragma unroll
                    for (int i = 0; i < kNdw; i++) cur[i] = nxt[i];
                }
                if (!hit) break;
                // rare: re-run step k exactly (the fast pass already left the end state)
                const int64_t c = c0 + kBlk * k;
                uint32_t prv[16];
                ld.load(c - 64, prv);
                const int64_t blo = lo - c, bhi = hi - c;
                const uint32_t idx = hash.exact(st0, prv, cur, blo < 0 ? 0 : static_cast<int>(blo),
                                                bhi > kBlk - 1 ? kBlk - 1 : static_cast<int>(bhi));
                if (idx < static_cast<uint32_t>(kBlk)) {
                    found = c + idx;
                    break;
                }
                if (++k >= nb) break;
                ld.load(c0 + kBlk * k, cur);
            }
        }
        const uint64_t hit = __ballot(found >= 0);
        if (hit) {
            const int first = __builtin_ctzll(hit);
            return static_cast<int64_t>(uni64(static_cast<uint64_t>(__shfl(found, first))));
        }
        ct += kWave * L;
    }
    return -1;
}

// ------------------------------------------------------------ batch kernel
struct BatchArgs {
    const uint8_t* const* ptrs;
    const uint64_t* lens;
    uint64_t* cuts;
    const uint64_t* cut_base;
    uint64_t* counts;
    uint32_t* queue;  // persistent-wave work counter (zeroed before each launch)
    // Time-sliced stream queue (LDS-DMA kernel): header words kQHead (tickets taken),
    // kQTail (streams yielded), kQDone (streams finished), kQErr (spin give-ups); ring[P]
    // holds {push number + 1, sid} of yielded streams (0 = empty; zeroed per launch, reset
    // on take).
    uint32_t* ring;
    uint64_t* help;       // help slots of the pipelined buzhash kernel (split_batch_pipe_kernel), else null
    uint32_t help_waves;  // launch waves = help slots
    uint32_t ring_mask;
    uint64_t* trace;  // KCDC_TRACE builds: 8 words per wave (split_batch_pipe_kernel) (else null)
    uint64_t cuts_cap;
    const uint64_t* cut_end;  // optional: stream i's cut range ends at cut_end[i] (else cut_base[i+1] / cuts_cap)
    const uint64_t* starts;   // optional: stream i's first chunk starts at starts[i] (else 0); the bytes before
                              // it are the window history of a continued stream (kcdc_bw_*)
    const uint64_t* resume;   // optional (with starts): the first chunk's test range resumes at resume[i]
    uint64_t min_size, max_size;
    const uint32_t* buz;
    const uint64_t* rk_out;
    const uint64_t* rk_mod;
    uint32_t nstreams;
    uint32_t mask;     // buzhash: the candidate mask in the rotated frame (below); rabin: as is
    uint32_t rk_shift;
    // buzhash rotated frame: the tables hold rotl(T, buz_rot), so every hash value is
    // rotl(H, buz_rot) and the test is (h & mask) == 0 with mask = rotl(avg - 1, buz_rot).
    // For avg a power of two buz_rot = 32 - log2(avg) moves the mask to the top bits and
    // "candidate" becomes h <= buz_lim (= ~mask): the hot loop's test is a bare v_min3.
    uint32_t buz_rot;
    uint32_t buz_lim;  // ~mask when mask is a top-bits mask (else unused)
    // Batch tiles: bytes per lane segment at most (a tile is 64 of them, ~avg/4): the scan of
    // a chunk's region stops at the tile holding its first candidate, and a tile of avg bytes
    // overshoots by ~58 % on average (exponential candidate gaps), one of avg/4 by ~13 %.
    uint32_t lane_cap;
    // Batch kernels: a region is published to helpers in windows of this many tiles (0:
    // the whole region).  Helpers claim a published window's tiles from its top down, so over a
    // whole region they scan its far end, which the owner's first candidate usually makes moot;
    // a window keeps them just ahead of the owner (re-published as the owner passes it).
    uint32_t help_window;
};

// End of stream sid's cut range (exclusive).
__device__ __forceinline__ uint64_t cut_end_of(const BatchArgs& a, uint32_t sid) {
    return a.cut_end ? a.cut_end[sid] : sid + 1 < a.nstreams ? a.cut_base[sid + 1] : a.cuts_cap;
}

template <int KIND>
struct HashSmem;
template <>
struct HashSmem<kBuzhash> {
    BuzShared s;
};
template <>
struct HashSmem<kRabinKarp> {
    RabinShared s;
};

template <int KIND>
__device__ __forceinline__ void fill_tables(HashSmem<KIND>& sm, const BatchArgs& a) {
    if constexpr (KIND == kBuzhash) {
        for (uint32_t i = threadIdx.x; i < 256u * 64u; i += blockDim.x) sm.s.tab[i] = rotl_n(a.buz[i >> 6], a.buz_rot);
    } else {
        for (uint32_t i = threadIdx.x; i < 256u; i += blockDim.x) {
            sm.s.out[i] = a.rk_out[i];
            sm.s.mod[i] = a.rk_mod[i];
        }
    }
    __syncthreads();
}

template <int KIND>
__device__ __forceinline__ auto make_hash(HashSmem<KIND>& sm, const BatchArgs& a, int lane) {
    if constexpr (KIND == kBuzhash) {
        BuzRing h;
        h.tab = reinterpret_cast<const char*>(sm.s.tab);
        h.lane4 = static_cast<uint32_t>(lane) * 4u;
        h.mask = a.mask;
        h.h = 0;
        return h;
    } else {
        Rabin h;
        h.tab = &sm.s;
        h.mask = a.mask;
        h.shift = a.rk_shift;
        h.v = 0;
        return h;
    }
}

// ------------------------------------------------ LDS-DMA fed batch path
// The per-lane 16-byte loads of scan_region() touch 64 different cache lines per instruction
// and are bound by the L1/L2 request rate, not HBM.  The batch and long-path kernels instead
// fetch every step by LDS-DMA (buffer_load_dwordx4 ... nt lds): each 128-byte line of a lane
// segment is one coalesced request (dma_step128), written to the wave's slot with a swizzle
// that keeps the ds_read_b128 lane groups conflict-free (read_step128).
#ifndef KCDC_TRACE
#define KCDC_TRACE 0  // timing-trace builds only (tools/trace_pipe.py)
#endif
// 8 waves x one 8 KiB step slot + 4 KiB warm slot (64 KiB table; 2 waves/SIMD, no VGPR spills):
// 4096 x 4 MiB 1.62 ms vs 12 waves 1.68, 7 waves 1.68 (round 1); deeper pipelines were slower
// (8 x 3 slots 1.68, 6 x 4 1.81, 4 x 6 2.00).
constexpr int kDmaWaves = 8;  // waves per workgroup (one workgroup per CU)
// Each step fetches 128 bytes (one whole cache line) of every lane segment, staged through
// ONE 8 KiB slot per wave: the step's bytes move to VGPRs at its start, which frees the
// slot for the next step's DMA while the step is hashed.
constexpr int kSlot = 64 * kWave;          // 4 KiB: one 64-byte piece of every lane (warm slot)
constexpr int kSlotBytes = 128 * kWave;    // 8 KiB: one 128-byte step of every lane
typedef __attribute__((address_space(3))) void* lds_ptr_t;

// The table and the DMA slots are SEPARATE __shared__ objects: LDS lowering then gives
// them distinct alias scopes, so the waitcnt pass knows a table read cannot alias an
// in-flight LDS-DMA into a slot.  In one struct every table read waited vmcnt(0) for the
// DMA just issued, which serialised the prefetch with the hashing.
struct DmaSlots {
    __attribute__((aligned(16))) uint8_t b[kDmaWaves][1][kSlotBytes];
};
constexpr int kRkWaves = kDmaWaves;  // waves per workgroup of the Rabin-Karp DMA kernels
struct RkSlots {
    __attribute__((aligned(16))) uint8_t b[kRkWaves][1][kSlotBytes];
};

// One LDS-DMA wave instruction (64 lanes x 16 B -> 1 KiB at LDS address m0), written as
// inline asm so the waitcnt pass does not see an LDS-DMA: with several DMA sites and slots
// it ran out of alias-tracking slots and made table reads wait vmcnt for in-flight slot
// fills.  Every slot read here is preceded by an explicit s_waitcnt; M0 is used by no other
// code in these kernels.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {  // LDS byte address of a __shared__ pointer
    return __builtin_amdgcn_readfirstlane(
        static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_ptr_t)(const_cast<void*>(p)))));
}
__device__ __forceinline__ void dma_lds16(const u32x4& d, uint32_t m0, int32_t voff) {
    // nt: the stream bytes are read once (membench: 128-B runs 6.65 vs 6.38 TB/s without it)
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen nt lds"
                 :: "s"(m0), "v"(voff), "s"(d) : "memory");
}

__device__ __forceinline__ void dma_piece(const Loader& ld, int64_t tb, uint32_t slot, int64_t ct,
                                          int64_t L, int64_t piece, int lane) {
    // descriptor offsets in 32 bits (ct - tb <= 64, a tile < 2^31 bytes): no per-lane 64-bit values
    const int32_t base = static_cast<int32_t>(ct - tb) + 64 * static_cast<int32_t>(piece), Li = static_cast<int32_t>(L);
    uint32_t sl = slot;  // opaque per call (as dma_step128): the m0 values are scalar adds, not spills
    asm volatile("" : "+s"(sl));
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int l = 16 * i + (lane >> 2);
        const int jj = (lane & 3) ^ ((l >> 2) & 3);
        dma_lds16(ld.d, sl + 1024u * i, base + l * Li + 16 * jj);
    }
}

__device__ __forceinline__ void read_piece(const uint8_t* slot, int lane, int64_t c, int64_t off0,
                                           uint32_t (&dw)[16]) {
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int q = 4 * lane + (j ^ ((lane >> 2) & 3));
        const u32x4 v = *reinterpret_cast<const u32x4*>(slot + 16 * q);
        dw[4 * j + 0] = v.x;
        dw[4 * j + 1] = v.y;
        dw[4 * j + 2] = v.z;
        dw[4 * j + 3] = v.w;
    }
    if (c == 0 && off0) {  // bytes before the stream start are virtual zeros
#pragma unroll
        for (int d = 0; d < 4; d++) {
            const int64_t keep_from = off0 - 4 * d;
            const uint32_t m = keep_from <= 0 ? 0xFFFFFFFFu
                                              : (keep_from >= 4 ? 0u : (0xFFFFFFFFu << (8 * keep_from)));
            dw[d] &= m;
        }
    }
}

// 128-byte runs: DMA lane d of instruction i (0..7) fetches chunk (d&7) ^ sw(l) of lane
// l = 8i + d/8, so lane l's line lands at slot + 128 l with chunk j at granule j ^ sw(l);
// sw(l) = (l >> 1) & 7 gives every ds_read_b128 lane group 16 distinct 16-byte bank slots.
__device__ __forceinline__ void dma_step128(const Loader& ld, int64_t tb, uint32_t slot, int64_t ct,
                                            int64_t L, int64_t n, int lane) {
    const int32_t base = static_cast<int32_t>(ct - tb) + 128 * static_cast<int32_t>(n), Li = static_cast<int32_t>(L);
    // the slot address made opaque per call: its eight m0 values are then one scalar add each,
    // not eight values kept across the hash loop (they were SGPR spills, a v_readlane per DMA)
    uint32_t sl = slot;
    asm volatile("" : "+s"(sl));
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const int l = 8 * i + (lane >> 3);
        const int jj = (lane & 7) ^ ((l >> 1) & 7);
        dma_lds16(ld.d, sl + 1024u * i, base + l * Li + 16 * jj);
    }
}

__device__ __forceinline__ void read_step128(const uint8_t* slot, int lane, int64_t c, int64_t off0,
                                             uint32_t (&dw)[32]) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const u32x4 v = *reinterpret_cast<const u32x4*>(slot + 128 * lane + 16 * (j ^ ((lane >> 1) & 7)));
        dw[4 * j + 0] = v.x;
        dw[4 * j + 1] = v.y;
        dw[4 * j + 2] = v.z;
        dw[4 * j + 3] = v.w;
    }
    if (c == 0 && off0) {  // bytes before the stream start are virtual zeros
#pragma unroll
        for (int d = 0; d < 4; d++) {
            const int64_t keep_from = off0 - 4 * d;
            const uint32_t m = keep_from <= 0 ? 0xFFFFFFFFu
                                              : (keep_from >= 4 ? 0u : (0xFFFFFFFFu << (8 * keep_from)));
            dw[d] &= m;
        }
    }
}

// The same with the head test precomputed (head: this lane's step starts at coordinate 0).
__device__ __forceinline__ void read_step128h(const uint8_t* slot, int lane, bool head, int64_t off0,
                                              uint32_t (&dw)[32]) {
    read_step128(slot, lane, head ? 0 : 1, off0, dw);
}

// Geometry of the tile starting at ct (lane segments of L bytes, nb 128-byte steps).
struct TileGeom {
    int64_t L;
    int nb;
    Loader ld;
};
__device__ __forceinline__ TileGeom tile_geom(int64_t ct, int64_t hi, const uint8_t* abase, int64_t off0,
                                              int64_t nbytes_coord, int64_t lane_cap = kLaneMax) {
    const int64_t rem = hi - ct + 1;
    int64_t per = (rem + kWave - 1) / kWave;
    per = (per + 127) & ~int64_t(127);
    TileGeom g;
    g.L = per < lane_cap ? per : lane_cap;
    g.nb = static_cast<int>(g.L / 128);
    g.ld = make_loader(abase, off0, nbytes_coord, ct >= 64 ? ct - 64 : 0);
    return g;
}

// Scan budget meaning "never yield" (a visit's quantum when no stream waits).
constexpr int64_t kNoYield = int64_t(1) << 62;

// ------------------------------------------- agent-scope atomics, queue header
typedef __attribute__((address_space(1))) uint32_t gu32;
typedef __attribute__((address_space(1))) uint64_t gu64;
__device__ __forceinline__ uint32_t ld_agent(uint32_t* p) {
    return __hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_agent64(uint64_t* p) {
    return __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent64(uint64_t* p, uint64_t v) {
    __hip_atomic_store((gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t add_agent(uint32_t* p, uint32_t v) {
    return __hip_atomic_fetch_add((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t bcast(uint32_t v) { return __builtin_amdgcn_readfirstlane(__shfl(v, 0)); }
__device__ __forceinline__ uint64_t bcast64(uint64_t v) {
    return (static_cast<uint64_t>(bcast(static_cast<uint32_t>(v >> 32))) << 32) | bcast(static_cast<uint32_t>(v));
}
// Header words (uint32 offsets) 2 KiB apart: hammered counters do not share DRAM pages.
// Word 0 holds the 64-bit {head, tail} ticket counter (kQHT, below).
constexpr int kQDone = 512, kQErr = 1536, kQSteal = 1024, kQHelp = 1600;
// Rarely read words (kept out of the kernel arguments, whose SGPRs the hot loop needs):
// kQCfg+0 spin cap, kQCfg+1 steal period; kQFlags.. one flag per workgroup (grid <= 256):
// 0 until workgroup b starts (1) or a waiting wave requeues its preassigned streams (2).
constexpr int kQCfg = 1040, kQFlags = 1088;
constexpr uint32_t kMaxPipeGrid = 256;
constexpr size_t kQHeaderBytes = 8192;
// Header words 1792.. : debug-build failure record (pcheck, KCDC_DEBUG_CHECKS).
[[maybe_unused]] constexpr int kQStat = 1792;
// Header words 1664.. : held-ticket audit (help tasks) -- [0] help tasks whose ticket register
// disagreed with the ticket's memory copy, [1] [2] the first such pair (register, memory);
// diagnostic builds (KCDC_HELP_DIAG) also [3] a bitmask of wave-uniform control values seen
// lane-divergent at the loop top and [4] the count of such observations.
constexpr int kQDiag = 1664;
// A waiting wave gives up (error word; a stream it held a ticket for is then reported failed)
// only after this many polls with no stream finishing: a bug guard that keeps the kernel
// bounded, >= 60 s; no correct launch waits that long (one wave scans >= 6 GB/s).
constexpr uint32_t kSpinCap = 1u << 26;
constexpr uint32_t kStealSpins = 256;                            // ~0.5 ms of polling between steal scans

// ======================================================= pipelined persistent kernel
// One per-wave state machine over tiles.  Every tile warms its 64 lanes on the 64 bytes
// before their segments (a 4 KiB piece in the wave's warm slot) and hashes 16 steps of
// 128-byte runs (8 KiB step slot).  The warm piece and first step of the NEXT tile are
// DMA'd during the current tile's last step, so a tile boundary exposes no latency:
//  * next tile of the same region: known in advance (the owner's claim on it, below);
//  * next stream (quantum spent, or the region's last tile with no further region): the
//    next ticket is taken by an atomic at the START of that tile and its ring entry
//    (progress + stream parameters, 7 tagged 16-byte sc1 granules) loaded mid-tile, so
//    both global round trips (~5 us each under full HBM load) hide under the hashing.
// Only a candidate that ends a region early (the next region is not known before the
// tile ends) and the first tile of the launch expose a DMA latency.
//
// Intra-region help (round 4).  At the end of a batch -- and in any launch with fewer streams
// than waves (a writer round, a handful of files) -- waves wait with nothing to scan while each
// remaining region is walked tile by tile by the one wave that owns its stream: launch time vs
// stream count (profiles/r04/tail) put that tail at ~0.2 ms of a 1.4 ms config-2 launch.
// cand(p) is a pure function of the 64 bytes ending at p, so any wave can scan
// any tile of a region; only the FIRST candidate decides the cut.  So every owner publishes its
// region in its help slot: the tile grid (tile 0 at ct0, T bytes per tile, K tiles, region end
// hi) and a claim word {epoch | top | bottom}.  The owner claims its tiles from the bottom (one
// atomic add per tile, issued a step ahead of need); a waiting wave claims the top tile by
// compare-and-swap, scans it as a one-tile task and posts the tile's first candidate, tagged with
// the slot's epoch, in the slot's result row.  An owner whose claim fails resolves the region
// from the row: the first candidate in tile order, else the forced cut; a row entry still pending
// after kHelpWaitTicks is scanned by the owner itself, so no owner depends on another wave.
constexpr int64_t kPipeYield = 768 << 10;  // visit quantum while streams wait (384 K-1.5 M: within noise)
constexpr int kPEntryLanes = 8;
constexpr int kPEntryStride = 128;

struct WarmSlots {
    __attribute__((aligned(16))) uint8_t b[kDmaWaves][kSlot];  // 4 KiB: the 64 bytes before each lane segment
};
static_assert(sizeof(DmaSlots) + sizeof(WarmSlots) + sizeof(BuzShared) <= 160 * 1024,
              "step slots + warm slots + table exceed the CU's 160 KiB of LDS");

struct PStream {
    uint32_t sid;    // | kHelpBit for a help task
    int64_t n, off0;
    const uint8_t* abase;
    uint64_t cb, cap, cnt;  // help task: cb = owner slot, cnt = tile index
    int64_t s, ct;          // chunk start (help task: the owner's tile 0); next tile coordinate (< 0: not set up)
    uint32_t epoch;         // help task: the owner slot's epoch
    int64_t aux;            // help task: the region end (coordinate)
};
constexpr uint32_t kHelpBit = 0x80000000u;

__device__ __forceinline__ void pstream_fresh(PStream& st, uint32_t sid, uint64_t p, uint64_t n, uint64_t cb,
                                              uint64_t cend) {
    st.sid = sid;
    st.n = static_cast<int64_t>(n);
    st.off0 = static_cast<int64_t>(p & 15u);
    st.abase = reinterpret_cast<const uint8_t*>(p - static_cast<uint64_t>(st.off0));
    st.cb = cb;
    st.cap = cend > cb ? cend - cb : 0;
    st.cnt = 0;
    st.s = 0;
    st.ct = -1;
    st.epoch = 0;
    st.aux = 0;
}

// Pin every field to a scalar register: the uniformity analysis otherwise loses track of
// values carried through the switch paths, and each LDS-DMA (its buffer descriptor must be
// scalar) then sits in a readfirstlane waterfall loop.
__device__ __forceinline__ void uniformize(PStream& st) {
    st.sid = __builtin_amdgcn_readfirstlane(st.sid);
    st.n = static_cast<int64_t>(uni64(static_cast<uint64_t>(st.n)));
    st.off0 = static_cast<int64_t>(uni64(static_cast<uint64_t>(st.off0)));
    st.abase = reinterpret_cast<const uint8_t*>(uni64(reinterpret_cast<uint64_t>(st.abase)));
    st.cb = uni64(st.cb);
    st.cap = uni64(st.cap);
    st.cnt = uni64(st.cnt);
    st.s = static_cast<int64_t>(uni64(static_cast<uint64_t>(st.s)));
    st.ct = static_cast<int64_t>(uni64(static_cast<uint64_t>(st.ct)));
    st.epoch = __builtin_amdgcn_readfirstlane(st.epoch);
    st.aux = static_cast<int64_t>(uni64(static_cast<uint64_t>(st.aux)));
}

__device__ __forceinline__ void emit_cut(const BatchArgs& a, PStream& st, int lane, int64_t v) {
    if (lane == 0 && st.cnt < st.cap) a.cuts[st.cb + st.cnt] = static_cast<uint64_t>(v);
    st.cnt++;
}

// Set up the next region to scan (chunks whose test range starts past the end are cut
// at once); returns false when the stream is finished (all cuts emitted).
__device__ __forceinline__ bool pstream_region(const BatchArgs& a, PStream& st, int lane) {
    while (st.ct < 0) {
        if (st.s >= st.n) return false;
        const int64_t pf = st.s + static_cast<int64_t>(a.min_size) - 1;
        if (pf >= st.n) {  // last chunk [s, n): nothing to test (splitter_buzhash32.go:29-40, 60-67)
            emit_cut(a, st, lane, st.n);
            st.s = st.n;
            return false;
        }
        st.ct = (pf + st.off0) & ~int64_t(127);
    }
    return true;
}

// First tile coordinate of stream e's first region when a previous round already tested the
// positions below resume[e] (kcdc_bw_*): the scan starts at the tile holding min(resume, region
// end) instead of at s + min - 1; -1 (set up as usual) otherwise.
__device__ __forceinline__ int64_t resume_ct(const BatchArgs& a, uint32_t e, int64_t s, int64_t n, int64_t off0) {
    if (!a.resume) return -1;
    const int64_t r = static_cast<int64_t>(a.resume[e]);
    const int64_t lo = s + static_cast<int64_t>(a.min_size) - 1;
    const int64_t mx = s + static_cast<int64_t>(a.max_size) - 1;
    const int64_t hi = mx < n - 1 ? mx : n - 1;
    if (lo > n - 1 || r <= lo) return -1;
    return ((r > hi ? hi : r) + off0) & ~int64_t(127);
}

// Ring entry of a yielded stream: granule l (< 7) = {tag, lo, hi, l == 0 ? sid : 0} of
// word l in {cnt, s, ct, ptr, n, cb, cap}.  Written by lane 0 alone (7 uniform 16-byte
// stores): a per-lane select chain over the words miscompiled (a word's high half read
// an undefined register).
__device__ __forceinline__ u32x4 pgranule(uint32_t tag, uint64_t w, uint32_t x) {
    u32x4 v;
    v.x = tag;
    v.y = static_cast<uint32_t>(w);
    v.z = static_cast<uint32_t>(w >> 32);
    v.w = x;
    return v;
}
// readlane returns int: widen through uint32_t, or a low word with bit 31 set sign-extends
// into the high word (it did: pointers came back as 0xFFFFFFFF'xxxxxxxx).
__device__ __forceinline__ uint64_t rl64(const u32x4& v, int l) {
    const uint32_t lo = static_cast<uint32_t>(__builtin_amdgcn_readlane(v.y, l));
    const uint32_t hi = static_cast<uint32_t>(__builtin_amdgcn_readlane(v.z, l));
    return (static_cast<uint64_t>(hi) << 32) | lo;
}
__device__ __forceinline__ void pentry_decode(PStream& st, const u32x4& v) {
    st.sid = __builtin_amdgcn_readlane(v.w, 0);
    st.cnt = rl64(v, 0);
    st.s = static_cast<int64_t>(rl64(v, 1));
    st.ct = static_cast<int64_t>(rl64(v, 2));
    const uint64_t p = rl64(v, 3);
    st.off0 = static_cast<int64_t>(p & 15u);
    st.abase = reinterpret_cast<const uint8_t*>(p - static_cast<uint64_t>(st.off0));
    st.n = static_cast<int64_t>(rl64(v, 4));
    st.cb = rl64(v, 5);
    st.cap = rl64(v, 6);
    st.aux = 0;
    st.epoch = 0;
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t pring_rsrc(const BatchArgs& a) {
    return __builtin_amdgcn_make_buffer_rsrc(a.ring, static_cast<short>(0),
                                             static_cast<int>((a.ring_mask + 1u) * kPEntryStride), 0x00020000);
}
// Every lane loads (lane & 7): no divergent load, so no copy of the result that would
// make the compiler wait for it early.
__device__ __forceinline__ u32x4 pentry_load(const BatchArgs& a, int lane, uint32_t e) {
    return __builtin_amdgcn_raw_buffer_load_b128(pring_rsrc(a),
                                                 static_cast<int>((e & a.ring_mask) * kPEntryStride) + 16 * (lane & 7), 0,
                                                 16 /* sc1 */);
}
__device__ __forceinline__ bool pentry_ok(const u32x4& v, int lane, uint32_t e) {
    return __ballot(lane < kPEntryLanes - 1 && v.x != e + 1u) == 0;
}

#ifndef KCDC_DEBUG_CHECKS
#define KCDC_DEBUG_CHECKS 0
#endif
// Debug builds: validate a resolved stream against the batch arrays; on a mismatch record
// {code, sid, ticket, detail} in header words kQStat+16.. and return false (wave exits).
__device__ __forceinline__ bool pcheck(const BatchArgs& a, int lane, const PStream& st, uint32_t tk, uint32_t where) {
#if KCDC_DEBUG_CHECKS
    if (st.sid & kHelpBit) return true;
    uint32_t code = 0;
    uint64_t detail = 0;
    const uint32_t sid = st.sid;
    if (sid >= a.nstreams) {
        code = 1;
        detail = st.sid;
    } else {
        const uint64_t p = uni64(reinterpret_cast<uint64_t>(a.ptrs[sid]));
        const uint64_t cb = uni64(a.cut_base[sid]);
        if (reinterpret_cast<uint64_t>(st.abase) + static_cast<uint64_t>(st.off0) != p) {
            code = 2;
            detail = reinterpret_cast<uint64_t>(st.abase);
        } else if (static_cast<uint64_t>(st.n) != uni64(a.lens[sid])) {
            code = 3;
            detail = static_cast<uint64_t>(st.n);
        } else if (st.cb != cb) {
            code = 4;
            detail = st.cb;
        } else if (st.cnt > st.cap) {
            code = 5;
            detail = st.cnt;
        } else if (st.cap != uni64(cut_end_of(a, sid)) - cb) {
            code = 7;
            detail = st.cap;
        } else if (st.s < 0 || st.s > st.n) {
            code = 6;
            detail = static_cast<uint64_t>(st.s);
        }
    }
    if (code) {
        if (lane == 0) {
            if (atomicAdd(a.queue + kQErr, 1u) == 0) {
                a.queue[kQStat + 16] = code | (where << 8);
                a.queue[kQStat + 17] = st.sid;
                a.queue[kQStat + 18] = tk;
                a.queue[kQStat + 19] = static_cast<uint32_t>(detail);
                a.queue[kQStat + 20] = static_cast<uint32_t>(detail >> 32);
                a.queue[kQStat + 21] = static_cast<uint32_t>(st.s);
                a.queue[kQStat + 22] = static_cast<uint32_t>(st.ct);
                a.queue[kQStat + 23] = static_cast<uint32_t>(st.cnt);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        return false;
    }
#endif
    return true;
}

// Queue counter: ONE 64-bit word {head = tickets taken (low), tail = entries reserved
// (high)} at header words 0..1, so a wave that yields one stream and takes the next does
// both with one atomic.  Entries 0..n-1 are the streams' initial states (init_ring_kernel
// writes them and sets tail = n); a reserved entry that ends up unused (its stream
// finished in the tile) is written as a tombstone (sid 0xFFFFFFFF), which a taker skips.
constexpr int kQHT = 0;
constexpr uint32_t kTombstone = 0xFFFFFFFFu;
__device__ __forceinline__ uint64_t qht_add(const BatchArgs& a, int lane, uint64_t inc) {
    uint64_t v = 0;
    if (lane == 0)
        v = __hip_atomic_fetch_add((gu64*)(reinterpret_cast<uint64_t*>(a.queue + kQHT)), inc, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
#if KCDC_DEBUG_CHECKS  // entries reserved (kQStat+32)
    if (lane == 0 && (inc >> 32)) add_agent(a.queue + kQStat + 32, static_cast<uint32_t>(inc >> 32));
#endif
    return v;  // lane 0's register
}
__device__ __forceinline__ uint64_t qht_value(uint32_t lo_raw, uint32_t hi_raw) {
    const uint32_t lo = static_cast<uint32_t>(__builtin_amdgcn_readlane(lo_raw, 0));
    const uint32_t hi = static_cast<uint32_t>(__builtin_amdgcn_readlane(hi_raw, 0));
    return (static_cast<uint64_t>(hi) << 32) | lo;
}
__device__ __forceinline__ uint64_t qht_take(const BatchArgs& a, int lane, uint64_t inc) {  // blocking
    const uint64_t raw = qht_add(a, lane, inc);
    return qht_value(static_cast<uint32_t>(raw), static_cast<uint32_t>(raw >> 32));
}

// Preassigned first tickets are spread over the grid: wave w of workgroup b holds ticket
// w * grid + b, so a launch with fewer streams than waves puts at most one owner on a CU (the
// others' SIMDs and DMA queues stay free for helpers).
__device__ __forceinline__ uint32_t first_ticket(uint32_t block, uint32_t wave) { return wave * gridDim.x + block; }

__device__ __forceinline__ void pwrite(const BatchArgs& a, int lane, uint32_t e, const PStream& st, bool tomb);

// Forward progress without co-residency.  Each wave's first ticket is preassigned
// (first_ticket, init_ring_kernel), so a workgroup that is not resident -- another kernel holds
// its CU -- would keep its streams while the resident waves wait for them.  A wave that has
// waited kStealSpins polls scans the workgroup flags; for a workgroup that has not started it
// swaps the flag 0 -> 2 and requeues that workgroup's preassigned streams as fresh ring
// entries (their initial states, rebuilt from the batch arrays).  A workgroup that starts
// later finds its flag at 2 and takes its tickets from the counter.  A waiting wave then
// waits only on entries reserved by running waves (written without blocking) or on streams
// held by running waves, so every wait ends.
__device__ bool try_steal(const BatchArgs& a, int lane, uint32_t wg_waves) {
    uint32_t found = 0xFFFFFFFFu;
    uint32_t* const flags = a.queue + kQFlags;
    const uint32_t nwg = gridDim.x;
    for (uint32_t b0 = 0; b0 < nwg; b0 += kWave) {
        const uint32_t b = b0 + static_cast<uint32_t>(lane);
        const uint32_t f = b < nwg ? ld_agent(flags + b) : 1u;
        const uint64_t m = __ballot(f == 0u);
        if (m) {
            found = b0 + static_cast<uint32_t>(__builtin_ctzll(m));
            break;
        }
    }
    found = __builtin_amdgcn_readfirstlane(found);
    if (found == 0xFFFFFFFFu) return false;
    uint32_t old = 1u;
    if (lane == 0) {
        old = 0u;
        __hip_atomic_compare_exchange_strong((gu32*)(flags + found), &old, 2u, __ATOMIC_RELAXED,
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (bcast(old) != 0u) return false;  // it started (or another wave stole it) meanwhile
    uint32_t k = 0;
    for (uint32_t w = 0; w < wg_waves; w++) k += first_ticket(found, w) < a.nstreams ? 1u : 0u;
    if (k == 0) return true;
    const uint64_t ht = qht_take(a, lane, static_cast<uint64_t>(k) << 32);  // reserve k entries
    const uint32_t e0 = static_cast<uint32_t>(ht >> 32);
    for (uint32_t w = 0; w < k; w++) {  // first_ticket grows with w: the first k waves held streams
        const uint32_t sid = first_ticket(found, w);
        PStream st;
        const uint64_t cb = uni64(a.cut_base[sid]);
        pstream_fresh(st, sid, uni64(reinterpret_cast<uint64_t>(a.ptrs[sid])), uni64(a.lens[sid]), cb,
                      uni64(cut_end_of(a, sid)));
        if (a.starts) st.s = static_cast<int64_t>(uni64(a.starts[sid]));
        st.ct = resume_ct(a, sid, st.s, st.n, st.off0);
        uniformize(st);
        pwrite(a, lane, e0 + w, st, false);
    }
    if (lane == 0) add_agent(a.queue + kQSteal, 1u);
    return true;
}

// ------------------------------------------------------------------ help slots
// Slot g (one per launch wave) in the help area: claim word at 128 * g (own line), the region
// granules at kHelpParams + 64 * g, the result row at kHelpRows + 8 * kHelpTiles * g, and bit g
// of the published-slots bitmap at kHelpBits (set while the region is open: waiting waves read
// the bitmap, then the claim words of set slots, instead of probing slots blindly).
//   claim  {epoch:24 | top:20 | bottom:20}: tiles [0, bottom) are the owner's, [top, K) the
//          helpers'; epoch 0 = nothing published (init_ring_kernel zeroes every claim word).
//   params 4 granules {epoch, lo, hi, x}: {ptr, sid}, {n, K}, {ct0, T}, {hi, 0}.
//   row[k] {epoch:24 | state:8 | rel:32}: state 1 no candidate in tile k, 2 first candidate at
//          ct0 + rel; anything else (or another epoch) pending.  Posted by atomic max, so a
//          stale helper's older epoch never overwrites a newer result.
#ifndef KCDC_HELP_EVERY
#define KCDC_HELP_EVERY 2
#endif
#ifndef KCDC_HELP_GAP  // a region is open to helpers while top >= bottom + GAP (1 vs 2: 1.295 vs
#define KCDC_HELP_GAP 1u  // 1.332 ms on config 2, same-process A/B, profiles/r04/third/)
#endif
#ifndef KCDC_HELP_MIN_AVG  // launch_split_batch's help policy: averages from here up (1 MiB)
#define KCDC_HELP_MIN_AVG (1ull << 20)
#endif
// Every region is published (a tail-only policy -- publish only in visits that began with no
// stream waiting -- lost 2-10 % at 1M-4M; DESIGN.md §2.1, profiles/r05/help_tail_only/).
__device__ __forceinline__ bool help_phase(int64_t budget) {
    (void)budget;
    return true;
}
constexpr int64_t kHelpSplit = 2;     // sub-tiles per help task (lane segments lane_cap / 2, >= 256 B)
constexpr int kHelpTiles = 128;          // regions of up to 128 tiles take help (every registered name)
#ifndef KCDC_HELP_MIN_TILES
#define KCDC_HELP_MIN_TILES 3u
#endif
constexpr uint32_t kHelpMinTiles = KCDC_HELP_MIN_TILES;  // the owner's tile, its next one, and at least one more
#ifndef KCDC_HELP_WAIT_TICKS
#define KCDC_HELP_WAIT_TICKS 20000
#endif
constexpr uint64_t kHelpWaitTicks = KCDC_HELP_WAIT_TICKS;  // 200 us of s_memrealtime (a tile takes 15-40 us)
__device__ __forceinline__ size_t help_params_off(uint32_t nw) { return 128ull * nw; }
__device__ __forceinline__ size_t help_rows_off(uint32_t nw) { return 128ull * nw + 64ull * nw; }
__device__ __forceinline__ size_t help_bits_off(uint32_t nw) { return help_rows_off(nw) + 8ull * kHelpTiles * nw; }
__device__ __forceinline__ uint32_t* help_bits(const BatchArgs& a) {
    return reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(a.help) + help_bits_off(a.help_waves));
}
__device__ __forceinline__ uint64_t* help_claim(const BatchArgs& a, uint32_t g) {
    return reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(a.help) + 128ull * g);
}
__device__ __forceinline__ uint64_t* help_row(const BatchArgs& a, uint32_t g) {
    return reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(a.help) + help_rows_off(a.help_waves)) +
           static_cast<uint64_t>(kHelpTiles) * g;
}
__device__ __forceinline__ uint64_t hclaim(uint32_t ep, uint32_t top, uint32_t bot) {
    return (static_cast<uint64_t>(ep) << 40) | (static_cast<uint64_t>(top) << 20) | bot;
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t help_params_rsrc(const BatchArgs& a) {
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<char*>(a.help) + help_params_off(a.help_waves),
                                             static_cast<short>(0), static_cast<int>(64u * a.help_waves), 0x00020000);
}

// Owner: publish region [ct0, hi] (K tiles of T bytes, tile 0 already the owner's) in slot g
// under epoch ep.  Order: the row zeroed and the granules stored write-through (sc1), drained,
// then the claim word -- a helper that sees epoch ep in the claim word reads granules and a row
// of that epoch (or of a later one, when the owner has moved on and waits for nothing).
__device__ void help_publish(const BatchArgs& a, int lane, uint32_t g, uint32_t ep, const PStream& st, int64_t ct0,
                             int64_t hi, uint32_t K, int64_t T) {
    uint64_t* row = help_row(a, g);
    for (uint32_t k = static_cast<uint32_t>(lane); k < K; k += kWave)
        __hip_atomic_store((gu64*)(row + k), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (lane == 0) {
        const __amdgpu_buffer_rsrc_t r = help_params_rsrc(a);
        const int base = static_cast<int>(64u * g);
        const uint64_t p = reinterpret_cast<uint64_t>(st.abase) + static_cast<uint64_t>(st.off0);
        __builtin_amdgcn_raw_buffer_store_b128(pgranule(ep, p, st.sid), r, base + 0, 0, 16 /* sc1 */);
        __builtin_amdgcn_raw_buffer_store_b128(pgranule(ep, static_cast<uint64_t>(st.n), K), r, base + 16, 0, 16);
        __builtin_amdgcn_raw_buffer_store_b128(pgranule(ep, static_cast<uint64_t>(ct0), static_cast<uint32_t>(T)), r,
                                               base + 32, 0, 16);
        __builtin_amdgcn_raw_buffer_store_b128(pgranule(ep, static_cast<uint64_t>(hi), 0), r, base + 48, 0, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) {
        __hip_atomic_store((gu64*)help_claim(a, g), hclaim(ep, K, 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_or((gu32*)(help_bits(a) + (g >> 5)), 1u << (g & 31u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
// Owner: no more tiles of this slot's region for helpers (the region or the visit ended).  The
// closed word carries the epoch with bit 23 set: claims of the open epoch fail, and a helper
// still scanning one of its tiles sees the change (every 4th step) and stops.
constexpr uint32_t kHelpClosed = 1u << 23;
__device__ __forceinline__ void help_close(const BatchArgs& a, int lane, uint32_t g, uint32_t ep) {
    if (lane == 0) {
        __hip_atomic_store((gu64*)help_claim(a, g), hclaim(ep | kHelpClosed, 0, 0), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_and((gu32*)(help_bits(a) + (g >> 5)), ~(1u << (g & 31u)), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
}
// Owner: read its claim word back by LDS-DMA (sc1, past L1) into LDS at m0 (16 bytes per lane,
// every lane the same granule: the word lands at m0).  The waitcnt pass does not see it (as the
// slot fills), so nothing waits for it inside the hash loop; the reader's own vmcnt wait does.
__device__ __forceinline__ void help_claim_dma(const BatchArgs& a, int lane, uint32_t g, uint32_t m0) {
    (void)lane;
    u32x4 d;
    const uint64_t base = reinterpret_cast<uint64_t>(a.help);
    d.x = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(base));
    d.y = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(base >> 32) & 0xFFFFu);
    d.z = __builtin_amdgcn_readfirstlane(128u * a.help_waves);
    d.w = 0x00020000u;
    const int32_t off = static_cast<int32_t>(128u * g);
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen sc1 lds"
                 :: "s"(m0), "v"(off), "s"(d) : "memory");
}
// Helper: post tile k's first candidate (coordinate f, or -1) to slot g's row under epoch ep.
__device__ __forceinline__ void help_post(const BatchArgs& a, int lane, uint32_t g, uint32_t ep, uint32_t k,
                                          int64_t ct0, int64_t f) {
    const uint64_t v = (static_cast<uint64_t>(ep) << 40) |
                       (f >= 0 ? (2ull << 32) | static_cast<uint64_t>(static_cast<uint32_t>(f - ct0)) : (1ull << 32));
    if (lane == 0) {
        __hip_atomic_fetch_max((gu64*)(help_row(a, g) + k), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        add_agent(a.queue + kQHelp, 1u);
    }
}
// The ticket a wave holds while it runs help tasks: kept in memory (word 2 of its help slot's
// claim line) from the moment the help task is taken, and taken back from there when the task
// ends, besides the copy in the task's cap field.  held_get audits the two (header words kQDiag..).
__device__ __forceinline__ void held_put(const BatchArgs& a, int lane, uint32_t me, uint32_t t) {
    if (lane == 0)
        __hip_atomic_store((gu64*)(help_claim(a, me) + 2), 0x100000000ull | t, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t held_get(const BatchArgs& a, int lane, uint32_t me, uint32_t reg) {
    const uint64_t raw = ld_agent64(help_claim(a, me) + 2);
    const uint32_t t = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(raw), 0));
    if (t != reg && lane == 0) {
        if (atomicAdd(a.queue + kQDiag, 1u) == 0) {
            a.queue[kQDiag + 1] = reg;
            a.queue[kQDiag + 2] = t;
        }
    }
    return t;  // always memory's copy: the register copy is only audited
}
#ifndef KCDC_HELP_DIAG
#define KCDC_HELP_DIAG 0
#endif
// Diagnostic builds: bit `bit` when v is not the same in every lane (a wave-uniform control value
// held lane-divergent).
__device__ __forceinline__ uint32_t divergent_bit(uint32_t v, int bit) {
    return __ballot(v != static_cast<uint32_t>(__shfl(static_cast<int>(v), 0))) != 0 ? 1u << bit : 0u;
}
__device__ __forceinline__ void diag_record(const BatchArgs& a, int lane, uint32_t bits) {
    if (bits && lane == 0) {
        atomicOr(a.queue + kQDiag + 3, bits);
        atomicAdd(a.queue + kQDiag + 4, 1u);
    }
}
// Owner whose claim failed: the helpers hold tiles [k0, K).  Returns the region's first
// candidate (coordinate) among them, -1 if they have none, or -2 - k when tile k is still
// pending after kHelpWaitTicks (the owner then scans from tile k itself).
__device__ int64_t help_wait(const BatchArgs& a, int lane, uint32_t g, uint32_t ep, uint32_t k0, uint32_t K,
                             int64_t ct0) {
    const uint64_t* row = help_row(a, g);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        int64_t res = -1;
        uint32_t pend_at = 0xFFFFFFFFu;
        for (uint32_t b = k0; b < K; b += kWave) {
            const uint32_t k = b + static_cast<uint32_t>(lane);
            const uint64_t v = k < K ? ld_agent64(const_cast<uint64_t*>(row + k)) : 0ull;
            const bool mine = k < K && static_cast<uint32_t>(v >> 40) == ep;
            const uint32_t stt = mine ? static_cast<uint32_t>(v >> 32) & 0xFFu : 0u;
            const uint64_t pend = __ballot(k < K && stt != 1u && stt != 2u);
            const uint64_t cand = __ballot(stt == 2u);
            const uint64_t ev = pend | cand;
            if (ev) {
                const int f = __builtin_ctzll(ev);
                if ((cand >> f) & 1ull) {
                    const uint32_t rel = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(v), f));
                    res = ct0 + static_cast<int64_t>(rel);
                } else {
                    pend_at = b + static_cast<uint32_t>(f);
                }
                break;
            }
        }
        if (pend_at == 0xFFFFFFFFu) return res;
        if (__builtin_amdgcn_s_memrealtime() - t0 > kHelpWaitTicks) return -2 - static_cast<int64_t>(pend_at);
        __builtin_amdgcn_s_sleep(8);
    }
}
// Waiting wave: claim the top tile of an open region with many unclaimed tiles.  The bitmap
// names the open slots; each lane takes one set bit of one bitmap word (words and bits start at
// positions that rotate with the wave and the attempt, so waiting waves spread over the owners),
// reads that slot's claim word, and the lane with the most unclaimed tiles (ties: rotated) tries
// the compare-and-swap.  On success `task` is a one-tile help task: sid | kHelpBit, the stream's
// pointer and length, s = the owner's tile 0, ct = the tile, aux = the tile's end, cb = slot,
// cnt = tile index, epoch.
__device__ bool help_find(const BatchArgs& a, int lane, uint32_t me, uint32_t attempt, PStream& task) {
    const uint32_t nw = a.help_waves, nwords = (nw + 31u) >> 5;
    const uint32_t rot = me * 7u + attempt * 13u;
    const uint32_t wi = (static_cast<uint32_t>(lane) + rot) % nwords;
    uint32_t bits = static_cast<uint32_t>(lane) < nwords ? ld_agent(help_bits(a) + wi) : 0u;
    if (wi == (me >> 5)) bits &= ~(1u << (me & 31u));  // not our own slot
    uint32_t g = 0xFFFFFFFFu;
    if (bits) {
        const uint32_t r = (rot >> 3) & 31u;
        const uint32_t rb = (bits >> r) | (r ? bits << (32u - r) : 0u);  // rotate right by r
        g = (wi << 5) + ((static_cast<uint32_t>(__builtin_ctz(rb)) + r) & 31u);
    }
    const uint64_t c = g < nw ? ld_agent64(help_claim(a, g)) : 0ull;
    const uint32_t ep = static_cast<uint32_t>(c >> 40), top = static_cast<uint32_t>(c >> 20) & 0xFFFFFu,
                   bot = static_cast<uint32_t>(c) & 0xFFFFFu;
    // claim only tiles >= bottom + KCDC_HELP_GAP - 1 (GAP 1: up to the owner's next tile, which the
    // owner then takes from the row instead of scanning it)
    const bool open = ep != 0u && !(ep & kHelpClosed) && top >= bot + KCDC_HELP_GAP;
    const uint32_t key = open ? ((top - bot) << 6) | ((static_cast<uint32_t>(lane) + rot) & 63u) : 0u;
    uint32_t best = key;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) best = max(best, static_cast<uint32_t>(__shfl_xor(static_cast<int>(best), d)));
    best = __builtin_amdgcn_readfirstlane(best);
    if (best == 0u) return false;
    const int f = __builtin_ctzll(__ballot(key == best));
    const uint32_t gs = static_cast<uint32_t>(__builtin_amdgcn_readlane(g, f));
    const uint64_t cw = (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(c >> 32), f)))
                         << 32) |
                        static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(c), f));
    uint64_t old = cw;
    if (lane == 0)
        __hip_atomic_compare_exchange_strong((gu64*)help_claim(a, gs), &old, cw - (1ull << 20), __ATOMIC_RELAXED,
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (qht_value(static_cast<uint32_t>(old), static_cast<uint32_t>(old >> 32)) != cw) return false;  // lost the race
    const uint32_t eps = static_cast<uint32_t>(cw >> 40);
    const uint32_t k = (static_cast<uint32_t>(cw >> 20) & 0xFFFFFu) - 1u;
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(help_params_rsrc(a), static_cast<int>(64u * gs) + 16 * (lane & 3),
                                                          0, 16 /* sc1 */);
    if (__ballot(lane < 4 && v.x != eps) != 0) return false;  // the owner has moved on: nobody waits for this tile
    const uint64_t p = rl64(v, 0);
    task.sid = static_cast<uint32_t>(__builtin_amdgcn_readlane(v.w, 0)) | kHelpBit;
    task.off0 = static_cast<int64_t>(p & 15u);
    task.abase = reinterpret_cast<const uint8_t*>(p - static_cast<uint64_t>(task.off0));
    task.n = static_cast<int64_t>(rl64(v, 1));
    task.s = static_cast<int64_t>(rl64(v, 2));  // tile 0
    const int64_t T = static_cast<int64_t>(static_cast<uint32_t>(__builtin_amdgcn_readlane(v.w, 2)));
    task.ct = task.s + static_cast<int64_t>(k) * T;
    const int64_t rhi = static_cast<int64_t>(rl64(v, 3));
    task.aux = task.ct + T - 1 < rhi ? task.ct + T - 1 : rhi;  // the tile's end
    task.cb = gs;
    task.cnt = k;
    task.cap = 0;
    task.epoch = eps;
    return true;
}

// Blocking resolution of ticket t (its ring entry, polled): 1 resolved, 2 tombstone (take
// another ticket), 3 a help task in st (the ticket is still held), 0 every stream is done, or
// the wave gave up (error word) -- it exits.
//   Polling backoff: in the tail ~1,000 waves poll their entry and the done counter; once 8 polls
//   in a row saw no stream finish they sleep s_sleep 32 (1.339-1.344 vs 1.363 ms on config 2,
//   profiles/r03/buz/kbench_poll_*.log) and read the done counter every 4th poll.
//   Help: a waiting wave looks for a tile to help with every kHelpEvery polls (help_find).
constexpr uint32_t kPollAfter = 8, kDoneEvery = 4, kHelpEvery = KCDC_HELP_EVERY;
__device__ int presolve(const BatchArgs& a, int lane, uint32_t t, PStream& st, uint32_t wg_waves, uint32_t me,
                        bool can_help) {
    const uint32_t n = a.nstreams;
    const uint32_t spin_cap = ld_agent(a.queue + kQCfg), steal_spins = ld_agent(a.queue + kQCfg + 1);
    uint32_t idle = 0;            // polls since a stream last finished
    uint32_t seen = ~0u;          // lane 0: streams done at the last poll
    for (uint32_t spin = 0;; spin++) {
        const u32x4 v = pentry_load(a, lane, t);
        if (pentry_ok(v, lane, t)) {
            if (static_cast<uint32_t>(__builtin_amdgcn_readlane(v.w, 0)) == kTombstone) return 2;
            pentry_decode(st, v);
            return 1;
        }
        uint32_t stop = 0;
        if (lane == 0 && spin % kDoneEvery == 0) {
            // Progress = streams finishing.  Not the {head, tail} word: every ticket take and
            // yield is an atomic on it, and waiting waves polling it slowed those by ~7%.
            const uint32_t done = ld_agent(a.queue + kQDone);
            idle = done == seen ? idle + 1 : 0;
            seen = done;
            if (done >= n) {
                stop = 1;
            } else if (idle + 1u >= spin_cap) {  // this poll included: a cap of 1 gives up at once (test knob)
                add_agent(a.queue + kQErr, 1u);
                // post-mortem (tools/batch_probe.py): the ticket this wave gave up on, in the spare
                // words of its help slot's claim line
                if (a.help && me < a.help_waves) help_claim(a, me)[1] = 0x100000000ull | t;
                stop = 1;
            }
        }
        if (bcast(stop)) return 0;
        if (steal_spins && spin % steal_spins == steal_spins - 1) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA is in flight here either
            try_steal(a, lane, wg_waves);
            continue;  // poll the entry again at once
        }
        if (can_help && spin % kHelpEvery == kHelpEvery - 1) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (help_find(a, lane, me, spin / kHelpEvery, st)) return 3;
        }
        // back off while nothing finishes: ~1,000 waiting waves polling two words every 0.5 us
        // load the L2 channel of the done counter in the batch's tail
        if (bcast(idle) >= kPollAfter)
            __builtin_amdgcn_s_sleep(32);
        else
            __builtin_amdgcn_s_sleep(16);
    }
}

// Write entry e (tag e + 1): the stream's state, or a tombstone.
__device__ __forceinline__ void pwrite(const BatchArgs& a, int lane, uint32_t e, const PStream& st, bool tomb) {
    const uint32_t tag = e + 1u;
    const uint64_t p = reinterpret_cast<uint64_t>(st.abase) + static_cast<uint64_t>(st.off0);
    const __amdgpu_buffer_rsrc_t r = pring_rsrc(a);
    const int base = static_cast<int>((e & a.ring_mask) * kPEntryStride);
#if KCDC_DEBUG_CHECKS  // entry writes (kQStat+33), and a slot written twice under one tag (code 9)
    if (lane == 0) {
        add_agent(a.queue + kQStat + 33, 1u);
        const u32x4 old = __builtin_amdgcn_raw_buffer_load_b128(r, base, 0, 16);
        const uint32_t ht_tail = ld_agent(a.queue + kQHT + 1);
        if ((old.x == tag || e >= ht_tail) && atomicAdd(a.queue + kQErr, 1u) == 0) {
            a.queue[kQStat + 16] = old.x == tag ? 9u : 10u;
            a.queue[kQStat + 17] = st.sid;
            a.queue[kQStat + 18] = e;
            a.queue[kQStat + 19] = ht_tail;
        }
    }
#endif
    if (lane == 0) {
        __builtin_amdgcn_raw_buffer_store_b128(pgranule(tag, st.cnt, tomb ? kTombstone : st.sid), r, base + 0, 0,
                                               16 /* sc1 */);
        __builtin_amdgcn_raw_buffer_store_b128(pgranule(tag, static_cast<uint64_t>(st.s), 0), r, base + 16, 0, 16);
        __builtin_amdgcn_raw_buffer_store_b128(pgranule(tag, static_cast<uint64_t>(st.ct), 0), r, base + 32, 0, 16);
        __builtin_amdgcn_raw_buffer_store_b128(pgranule(tag, p, 0), r, base + 48, 0, 16);
        __builtin_amdgcn_raw_buffer_store_b128(pgranule(tag, static_cast<uint64_t>(st.n), 0), r, base + 64, 0, 16);
        __builtin_amdgcn_raw_buffer_store_b128(pgranule(tag, st.cb, 0), r, base + 80, 0, 16);
        __builtin_amdgcn_raw_buffer_store_b128(pgranule(tag, st.cap, 0), r, base + 96, 0, 16);
    }
}

// Mid-tile fetch of ring entry e by LDS-DMA (sc1) into the wave's warm slot, which is idle
// between the tile's warm-up and its last step; read back after the last step's explicit
// vmcnt wait.  A compiler-visible load instead would be in flight when the step's
// (inline-asm, invisible) LDS-DMAs issue, and the waitcnt pass would then put a vmcnt
// wait into the hash loop that also drains those DMAs.
__device__ __forceinline__ void pentry_dma(const BatchArgs& a, int lane, uint32_t e, uint32_t m0) {
    u32x4 d;
    const uint64_t base = reinterpret_cast<uint64_t>(a.ring);
    d.x = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(base));
    d.y = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(base >> 32) & 0xFFFFu);
    d.z = __builtin_amdgcn_readfirstlane((a.ring_mask + 1u) * kPEntryStride);
    d.w = 0x00020000u;
    const int32_t off = static_cast<int32_t>((e & a.ring_mask) * kPEntryStride) + 16 * (lane & 7);
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen sc1 lds"
                 :: "s"(m0), "v"(off), "s"(d) : "memory");
}

// Region bounds (coordinates) of the stream's current chunk; a help task's is its tile
// [ct, region end].
__device__ __forceinline__ void pregion(const BatchArgs& a, const PStream& st, int64_t& lo, int64_t& hi) {
    if (st.sid & kHelpBit) {
        lo = st.ct;
        hi = st.aux;
        return;
    }
    const int64_t mn = static_cast<int64_t>(a.min_size), mx = static_cast<int64_t>(a.max_size);
    lo = st.s + mn - 1 + st.off0;
    hi = (st.s + mx - 1 < st.n - 1 ? st.s + mx - 1 : st.n - 1) + st.off0;
}

__device__ __forceinline__ void ptile_issue(const PStream& st, int64_t hi, uint32_t wl, uint32_t sl, int lane,
                                            int64_t lane_cap) {
    const TileGeom g = tile_geom(st.ct, hi, st.abase, st.off0, st.off0 + st.n, lane_cap);
    dma_piece(g.ld, g.ld.tb, wl, st.ct, g.L, -1, lane);
    dma_step128(g.ld, g.ld.tb, sl, st.ct, g.L, 0, lane);
}

// Visit quantum from the number of streams queued behind the taken ticket: none waiting ->
// run to completion; otherwise 768 KiB (short tail quanta measured no gain, and helpers now
// split the tail's regions).
__device__ __forceinline__ int64_t pipe_quantum(int64_t backlog, int64_t q = kPipeYield) { return backlog <= 0 ? kNoYield : q; }
// The buzhash kernel's quantum in tiles: 6 full tiles, at least 512 KiB.  4M and larger averages
// keep 6 x 128 KiB = 768 KiB (512 KiB there: 1.334 vs 1.286 ms); 128K and 256K get 512 KiB.  Against
// the constant 768 KiB in one process (profiles/r04/third/ab_quantum_tiles_*.log): 128K 3.415 vs
// 3.639 ms, 256K 2.697 vs 2.843, 4M 1.296 vs 1.309; all bit-exact.
#ifndef KCDC_QUANTUM_TILES
#define KCDC_QUANTUM_TILES 6
#endif
__device__ __forceinline__ int64_t pipe_quantum_tiles(int64_t backlog, uint32_t lane_cap) {
    constexpr int64_t kTiles = KCDC_QUANTUM_TILES, kMax = kTiles * kWave * 2048;  // (2 KiB lanes: 768 KiB)
    const int64_t q = kTiles * kWave * static_cast<int64_t>(lane_cap);
    return pipe_quantum(backlog, q < (512 << 10) ? (512 << 10) : q > kMax ? kMax : q);
}

template <bool TOP>
__global__ __launch_bounds__(kDmaWaves * kWave, kDmaWaves / 4) void split_batch_pipe_kernel(BatchArgs a) {
    __shared__ BuzShared smtab;
    __shared__ DmaSlots smslots;
    __shared__ WarmSlots smwarm;
    fill_buz_table(smtab, a.buz, a.buz_rot);
    __syncthreads();
    const int lane = threadIdx.x & (kWave - 1);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const uint32_t me = blockIdx.x * kDmaWaves + wave;  // this wave's help slot
    BuzRing hash;
    hash.tab = reinterpret_cast<const char*>(smtab.tab);
    hash.lane4 = static_cast<uint32_t>(lane) * 4u;
    hash.mask = a.mask;
    hash.h = 0;
    uint8_t* sl = smslots.b[wave][0];
    uint8_t* wl = smwarm.b[wave];
    const uint32_t sl32 = lds_addr(sl), wl32 = lds_addr(wl);
#if KCDC_TRACE  // per wave at trace[8 * global wave]: start, end, ticks in blocking takes, the last take's
                // start, help tiles, their ticks, the end of the wave's last own tile, own tiles
    const uint32_t gw = blockIdx.x * kDmaWaves + wave;
    uint64_t tr_block = 0, tr_nblock = 0, tr_last = 0, tr_help = 0, tr_help_t = 0, tr_own_end = 0, tr_own = 0;
    if (lane == 0) a.trace[8 * gw] = __builtin_amdgcn_s_memrealtime();
#define KCDC_PRET                                                                 \
    do {                                                                          \
        if (lane == 0) {                                                          \
            a.trace[8 * gw + 1] = __builtin_amdgcn_s_memrealtime();                \
            a.trace[8 * gw + 2] = tr_block;                                       \
            a.trace[8 * gw + 3] = tr_last;                                        \
            a.trace[8 * gw + 4] = tr_help;                                        \
            a.trace[8 * gw + 5] = tr_help_t;                                      \
            a.trace[8 * gw + 6] = tr_own_end;                                     \
            a.trace[8 * gw + 7] = tr_own;                                         \
        }                                                                         \
        return;                                                                   \
    } while (0)
#else
#define KCDC_PRET return
#endif
    const uint32_t lim = TOP ? a.buz_lim : 0u;
    const int64_t mx = static_cast<int64_t>(a.max_size);
    // help sub-tiles halve the lane segments (>= 256 B): shift = sid's help bit & this (integer
    // arithmetic: a select on a bool here became a VALU-materialised shift next to the DMAs)
    const uint32_t help_shift = __builtin_amdgcn_readfirstlane(a.lane_cap >= 512u ? 1u : 0u);
    static_assert(kHelpSplit == 2, "help sub-tiles: one halving");

    PStream cur;
    int64_t budget = kNoYield;
    // Help state of this wave's own slot (wave-uniform, packed: SGPRs are what this kernel runs
    // short of): hep = the epoch of the last publish; hs = the published region's tile count
    // (bits 0-7), the index of the tile being scanned (8-15) and the flags below.
    uint32_t hep = 0, hs = 0;
    constexpr uint32_t kHsPub = 1u << 16;     // the current region is published (claims are on)
    constexpr uint32_t kHsNeedPub = 1u << 17; // the region at cur.ct is new to this wave
    constexpr uint32_t kHsHelped = 1u << 18;  // the last claim saw helpers on the region: no yield
    hs = kHsNeedPub;
    auto hK = [&] { return hs & 0xFFu; };
    auto htile = [&] { return (hs >> 8) & 0xFFu; };
    // Blocking take of the next stream with a region to scan (t: a ticket already held,
    // or ~0u to take one); false when every stream is done.  No LDS-DMA may be in flight.
    // claim: the first take's claim of this workgroup's preassigned tickets (lane 0's CAS
    // result: 0 or 1 ours, 2 the streams were requeued by try_steal), issued before the first
    // resolve and checked after it so its round trip overlaps the entry load; ~0u elsewhere
    // (a constant at those call sites: no claim state stays live across the main loop).
    auto take_blocking = [&](uint32_t t, int64_t backlog_hint, uint32_t claim) -> bool {
#if KCDC_TRACE
        const uint64_t tb0 = __builtin_amdgcn_s_memrealtime();
        tr_last = tb0;
        struct Acc {
            uint64_t t0, &sum, &cnt;
            __device__ ~Acc() {
                sum += __builtin_amdgcn_s_memrealtime() - t0;
                cnt++;
            }
        } acc{tb0, tr_block, tr_nblock};
#endif
        for (;;) {
            int64_t backlog = backlog_hint;  // queue depth behind a ticket already held (caller's estimate)
            if (t == 0xFFFFFFFFu) {
                const uint64_t ht = qht_take(a, lane, 1);
                t = static_cast<uint32_t>(ht);
                backlog = static_cast<int64_t>(ht >> 32) - static_cast<int64_t>(t) - 1;
            }
            const uint32_t held = t;
            const int r = presolve(a, lane, held, cur, kDmaWaves, me, a.help != nullptr && claim == 0xFFFFFFFFu);
            if (r == 0) return false;
            if (r == 3) {  // a help task; the ticket stays held (in cap, unused by help tasks, and in memory)
                held_put(a, lane, me, held);
                cur.cap = held;
                uniformize(cur);
                return true;
            }
            t = 0xFFFFFFFFu;
            if (claim != 0xFFFFFFFFu) {
                const bool requeued = bcast(claim) == 2u;
                claim = 0xFFFFFFFFu;
                if (requeued) continue;  // requeued by another wave: take a fresh ticket
            }
            if (r == 2) continue;  // tombstone
            uniformize(cur);
            if (!pcheck(a, lane, cur, held, 1)) return false;
            budget = pipe_quantum_tiles(backlog, a.lane_cap);
            if (pstream_region(a, cur, lane)) return true;
            if (lane == 0) {  // nothing left to scan
                a.counts[cur.sid] = cur.cnt;
                add_agent(a.queue + kQDone, 1u);
            }
        }
    };
    // Pending blocking take (set right before jumping to the loop top, so none of it is live
    // across the hash loop).
    bool need_take = true;
    uint32_t take_t = 0xFFFFFFFFu, take_claim = 0xFFFFFFFFu;
    int64_t take_backlog = 0;
    {
        // First ticket: preassigned (see init_ring_kernel), unless a waiting wave has requeued
        // this workgroup's streams before it started (try_steal): then take one from the counter.
        uint32_t claim = 1u;
        if (lane == 0) {
            claim = 0u;
            __hip_atomic_compare_exchange_strong((gu32*)(a.queue + kQFlags + blockIdx.x), &claim, 1u,
                                                 __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        const uint32_t t0 = first_ticket(blockIdx.x, wave);
        const int64_t nw = static_cast<int64_t>(gridDim.x) * kDmaWaves;
        take_t = t0 < a.nstreams ? t0 : 0xFFFFFFFFu;
        take_backlog = static_cast<int64_t>(a.nstreams) - nw;
        take_claim = t0 < a.nstreams ? (claim & 3u) : 0xFFFFFFFFu;
    }
    bool issued = false;  // this tile's warm piece + step 0 are in flight
    for (;;) {
#if KCDC_HELP_DIAG
        diag_record(a, lane, divergent_bit(need_take, 0) | divergent_bit(take_t, 1) | divergent_bit(issued, 2));
#endif
        // The one blocking take site (inlined once: presolve and try_steal are large).
        if (need_take) {
            if (!take_blocking(take_t, take_backlog, take_claim)) KCDC_PRET;
            need_take = false;
            issued = false;
            hs |= kHsNeedPub;
        }
#if KCDC_HELP_DIAG
        diag_record(a, lane, divergent_bit(hs, 3) | divergent_bit(hep, 4) | divergent_bit(cur.sid, 5) |
                                 divergent_bit(static_cast<uint32_t>(cur.cap), 6) |
                                 divergent_bit(static_cast<uint32_t>(cur.ct), 7) |
                                 divergent_bit(static_cast<uint32_t>(budget), 8));
#endif
        uniformize(cur);
        if (!pcheck(a, lane, cur, 0xFFFFFFFFu, 5)) return;
        const bool is_help = (cur.sid & kHelpBit) != 0;
#if KCDC_TRACE
        const uint64_t tr_t0 = __builtin_amdgcn_s_memrealtime();
        if (is_help) tr_help++;
        else tr_own++;
#endif
        int64_t lo, hi;
        pregion(a, cur, lo, hi);
        // A help task's tile (one owner tile, up to hi) goes in kHelpSplit sub-tiles: it stops at
        // the first one with a candidate, or when its owner has closed the region meanwhile.
        const int64_t lcap = static_cast<int64_t>(a.lane_cap >> ((cur.sid >> 31) & help_shift));
        const TileGeom g = tile_geom(cur.ct, hi, cur.abase, cur.off0, cur.off0 + cur.n, lcap);
        const int64_t ct = cur.ct, ct_next = ct + kWave * g.L;
        const bool last_of_region = ct_next > hi;
        if (!issued) ptile_issue(cur, hi, wl32, sl32, lane, lcap);
        // A region new to this wave: publish it when it is long enough to share.
        if ((hs & kHsNeedPub) && !is_help) {
            const int64_t T = kWave * static_cast<int64_t>(a.lane_cap);  // bytes per full tile
            const uint32_t K = static_cast<uint32_t>((hi - ct + T) / T);
            hs = 0;
            if (a.help && help_phase(budget) && K >= kHelpMinTiles && K <= static_cast<uint32_t>(kHelpTiles)) {
                // a window of the region (help_window tiles from here), re-published as the owner
                // passes its end
                const uint32_t Kw = a.help_window && K > a.help_window ? a.help_window : K;
                hep++;
                hs = kHsPub | Kw;
                help_publish(a, lane, me, hep, cur, ct, Kw < K ? ct + static_cast<int64_t>(Kw) * T - 1 : hi, Kw, T);
            }
        }
        // The owner's claim on its next tile (atomic add on its slot's bottom), issued in step 0
        // behind the refill DMA and read in step 2 (or at the tile end for one- and two-step tiles).
        const bool claim_next_r = (hs & kHsPub) && !is_help && !last_of_region && htile() + 1u < hK();
        // (a help task never yields: its wave's budget is the last own visit's leftover, and a
        // reservation made here would never be written -- its ticket's taker would wait to the end)
        const bool budget_out = !is_help && !(hs & kHsHelped) && budget - kWave * g.L <= 0;  // (with helpers: no yield)
        bool ends_nocand = false;  // no candidate in this tile => the stream is finished
        if (!is_help && last_of_region) {
            const int64_t s2 = cur.s + mx - 1 <= cur.n - 1 ? cur.s + mx : cur.n;
            ends_nocand = s2 >= cur.n || s2 + static_cast<int64_t>(a.min_size) - 1 >= cur.n;
        }
        // The visit's last tile (absent a candidate): take the next ticket now, and reserve
        // this stream's entry too when it will be yielded -- one atomic, hidden by the DMAs.
        const bool switching = !is_help && (budget_out || ends_nocand);
        const bool reserve = budget_out && !ends_nocand;
        const bool claim_next = claim_next_r && !switching;  // a yielding owner claims nothing more
        uint64_t ht_raw = 0;
        if (switching) ht_raw = qht_add(a, lane, 1);  // the next stream's ticket
        // Lane positions as 32-bit offsets from the tile start (a tile < 2^31 bytes): 64-bit
        // per-lane values live across the hash loop cost VGPRs this kernel does not have.
        const int32_t cl0 = lane * static_cast<int32_t>(g.L);
        const int32_t hi_rel = static_cast<int32_t>(hi - ct < 0x7FFFFFFF ? hi - ct : 0x7FFFFFFF);
        uint32_t ht_lo = static_cast<uint32_t>(ht_raw), ht_hi = static_cast<uint32_t>(ht_raw >> 32);
        {
            uint32_t w16[16];
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_waitcnt vmcnt(0)" : "+v"(ht_lo), "+v"(ht_hi)::"memory");
            read_piece(wl, lane, 1, cur.off0, w16);  // (the piece before coordinate 0 reads as zeros)
            hash.clear();
            hash.template block<kWarm>(w16);
        }
        uint32_t tk = 0;
        int64_t nbacklog = 0;
        if (switching) {
            const uint64_t ht = qht_value(ht_lo, ht_hi);
            tk = static_cast<uint32_t>(ht);
            nbacklog = static_cast<int64_t>(ht >> 32) + (reserve ? 1 : 0) - static_cast<int64_t>(tk) - 1;
        }
        uint64_t pe_raw = 0;
        bool res_issued = false;
        int nstate = 0;  // 0: next stream unresolved, 2: resolved, 3: + its first tile prefetched
        PStream nx;
        nx.ct = -1;
        bool next_issued = false;
        int32_t found = -1;  // offset from ct of this lane's first candidate
        const int poll_step = g.nb > 1 ? g.nb / 2 : 0;
        // The owner's claim on tile htile + 1: an atomic add on its slot's bottom in step 0 (no
        // return value: nothing stays live across the hashing), the word read back by an sc1
        // LDS-DMA into the idle warm slot in step 1 (behind step 1's wait, which the add has
        // passed) and looked at in the last step, before the next tile's prefetch.  One- and
        // two-step tiles read it at the tile end (and prefetch nothing).
        bool claim_ok = false, claim_known = !claim_next;
        auto claim_decode = [&](uint64_t cw) {  // cw: the claim word after this tile's add
            const uint32_t top = static_cast<uint32_t>(cw >> 20) & 0xFFFFFu, bot = static_cast<uint32_t>(cw) & 0xFFFFFu;
            claim_ok = static_cast<uint32_t>(cw >> 40) == hep && bot <= top;
            if (top < hK()) hs |= kHsHelped;
            claim_known = true;
        };
        for (int n = 0; n < g.nb; n++) {
            const int32_t cl = cl0 + 128 * n;
            const uint32_t st0 = hash.save();
            uint32_t dw[32];
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            read_step128h(sl, lane, ct == 0 && cl == 0, cur.off0, dw);
            if (claim_next && n >= 2 && n == g.nb - 1) claim_decode(*reinterpret_cast<const uint64_t*>(wl));
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot free: refill it
            __builtin_amdgcn_sched_barrier(0);

            if (reserve && n == g.nb - 1) {  // this stream's entry, reserved late
                pe_raw = qht_add(a, lane, 1ull << 32);
                res_issued = true;
            }
            if (switching && n == poll_step) {
                pentry_dma(a, lane, tk, wl32);
                if (n == g.nb - 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // nothing to hide it under
            }
            if (claim_next && n == 1) help_claim_dma(a, lane, me, wl32);
            if (n + 1 < g.nb) {
                dma_step128(g.ld, g.ld.tb, sl32, ct, g.L, n + 1, lane);
            } else if (!switching && !last_of_region && claim_known && (!claim_next || claim_ok) &&
                       __ballot(found >= 0) == 0) {
                // (a candidate in an earlier step means the region's cut is in this tile: the
                // next tile would be a stale prefetch, 12 KiB of HBM traffic per chunk wasted --
                // 9 % of R at 128K, where chunks span ~4 tiles)
                PStream t2 = cur;  // next tile of this region (ours)
                t2.ct = ct_next;
                ptile_issue(t2, hi, wl32, sl32, lane, lcap);
                next_issued = true;
            }
            if (claim_next && n == 0 && lane == 0)
                __hip_atomic_fetch_add((gu64*)help_claim(a, me), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __builtin_amdgcn_sched_barrier(0);
            const uint32_t m = hash.template step128<TOP>(dw, 0u);
            __builtin_amdgcn_sched_barrier(0);
            if (m <= lim && found < 0 && cl <= hi_rel) {  // rare: exact re-run from global memory
                const int64_t c = ct + cl;
                uint32_t prv[16], cur32[32];
                g.ld.load(c - 64, prv);
                g.ld.load(c, cur32);
                const int64_t blo = lo - c, bhi = hi - c;
                const uint32_t idx = hash.exact(st0, prv, cur32, blo < 0 ? 0 : static_cast<int>(blo),
                                                bhi > 127 ? 127 : static_cast<int>(bhi));
                if (idx < 128u) found = cl + static_cast<int32_t>(idx);
                // a wait the waitcnt pass sees: its scoreboard otherwise keeps these loads
                // pending around the loop and waits for them in the hash loop (draining DMAs)
                __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
            }
        }
        // ---- end of tile
        if (!claim_known) {  // a one- or two-step tile: its claim is read here
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (g.nb == 2) {
                claim_decode(*reinterpret_cast<const uint64_t*>(wl));
            } else {
                const uint64_t raw = ld_agent64(help_claim(a, me));
                claim_decode(qht_value(static_cast<uint32_t>(raw), static_cast<uint32_t>(raw >> 32)));
            }
        }
        if (reserve && !res_issued) {
            pe_raw = qht_add(a, lane, 1ull << 32);
            res_issued = true;
        }
        const uint64_t hit = __ballot(found >= 0);
#if KCDC_TRACE
        if (is_help) tr_help_t += __builtin_amdgcn_s_memrealtime() - tr_t0;
        else tr_own_end = __builtin_amdgcn_s_memrealtime();
#endif
        if (is_help) {
            bool done = true;
            if (hit || last_of_region) {  // post the tile's first candidate to its owner's row
                int64_t f = -1;
                if (hit) f = ct + __builtin_amdgcn_readfirstlane(__shfl(found, __builtin_ctzll(hit)));
                help_post(a, lane, static_cast<uint32_t>(cur.cb), cur.epoch, static_cast<uint32_t>(cur.cnt), cur.s, f);
            } else {  // the next sub-tile (prefetched), unless the owner has closed the region
                const uint64_t w = ld_agent64(help_claim(a, static_cast<uint32_t>(cur.cb)));
                done = static_cast<uint32_t>(qht_value(static_cast<uint32_t>(w), static_cast<uint32_t>(w >> 32)) >> 40) !=
                       cur.epoch;
            }
            if (!done) {
                cur.ct = ct_next;
                issued = next_issued;
                continue;
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the post, or a dropped prefetch
            need_take = true;
            take_t = held_get(a, lane, me, static_cast<uint32_t>(cur.cap));
            take_backlog = 0;
            take_claim = 0xFFFFFFFFu;
            continue;
        }
        bool region_changed = true;
        const int64_t forced = cur.s + mx - 1 <= cur.n - 1 ? cur.s + mx : cur.n;  // max-size cut / the end
        int64_t cut = -1;  // this region's cut, once known
        if (hit) {
            const int64_t f = ct + __builtin_amdgcn_readfirstlane(__shfl(found, __builtin_ctzll(hit)));
            cut = f - cur.off0 + 1;
        } else if (last_of_region) {  // forced cut at max size (splitter_buzhash32.go:60-64) or the end
            cut = forced;
        } else if (claim_next && !claim_ok) {  // the helpers hold the rest of the region
            const int64_t T = kWave * static_cast<int64_t>(a.lane_cap);
            const int64_t ct0 = ct - static_cast<int64_t>(htile()) * T;  // the published tile 0
            const int64_t r = help_wait(a, lane, me, hep, htile() + 1u, hK(), ct0);
            const int64_t wend = ct0 + static_cast<int64_t>(hK()) * T;  // past the published window
            if (r >= 0) {
                cut = r - cur.off0 + 1;
            } else if (r == -1 && wend <= hi) {  // no candidate in the window: publish the next one
                cur.ct = wend;
                help_close(a, lane, me, hep);
                hs = kHsNeedPub;
                region_changed = false;
            } else if (r == -1) {
                cut = forced;
            } else {  // a tile still pending: scan on from it, unshared
                cur.ct = ct0 + (-2 - r) * T;
                help_close(a, lane, me, hep);
                hs = 0;
                region_changed = false;
            }
        } else {
            cur.ct = ct_next;
            hs += 1u << 8;  // htile++
            budget -= kWave * g.L;
            region_changed = false;
            if ((hs & kHsPub) && htile() >= hK()) {  // past its published window: the next one
                help_close(a, lane, me, hep);
                hs = kHsNeedPub;
            }
        }
        if (cut >= 0) {
            emit_cut(a, cur, lane, cut);
            cur.s = cut;
            cur.ct = -1;
        }
        if (region_changed) {
            if (hs & kHsPub) help_close(a, lane, me, hep);
            hs = kHsNeedPub;
        }
        const bool live = pstream_region(a, cur, lane);
        if (!live && lane == 0) {
            a.counts[cur.sid] = cur.cnt;
            add_agent(a.queue + kQDone, 1u);
        }
        if (!switching && live) {  // same stream, next tile
            issued = next_issued && !region_changed;
            if (next_issued && region_changed) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // stale prefetch
            continue;
        }
        // ---- switch streams: requeue this one first (its reserve atomic was issued in the
        // last step, so no prefetch DMA is in flight behind it), then prefetch the next
        if (hs & kHsPub) help_close(a, lane, me, hep);  // a yielded region is not ours to share any more
        hs = kHsNeedPub;
        if (reserve) {
            const uint32_t pe = static_cast<uint32_t>(
                qht_value(static_cast<uint32_t>(pe_raw), static_cast<uint32_t>(pe_raw >> 32)) >> 32);
            pwrite(a, lane, pe, cur, !live);
        } else if (live) {  // a candidate kept the stream alive past its predicted last tile
            const uint64_t ht = qht_take(a, lane, 1ull << 32);
            pwrite(a, lane, static_cast<uint32_t>(ht >> 32), cur, false);
        }
        if (switching) {  // next stream: its entry landed in the warm slot (the last step's wait drained it)
            const u32x4 ev = *reinterpret_cast<const u32x4*>(wl + 16 * (lane & 7));
            if (pentry_ok(ev, lane, tk) && static_cast<uint32_t>(__builtin_amdgcn_readlane(ev.w, 0)) != kTombstone) {
                pentry_decode(nx, ev);
                uniformize(nx);
                if (!pcheck(a, lane, nx, tk, 2)) return;
                nstate = 2;
                if (nx.ct < 0 && nx.s < nx.n && nx.s + static_cast<int64_t>(a.min_size) - 1 < nx.n)
                    nx.ct = (nx.s + static_cast<int64_t>(a.min_size) - 1 + nx.off0) & ~int64_t(127);
                if (nx.ct >= 0) {  // prefetch its first tile now, under this tile's bookkeeping
                    int64_t nlo, nhi;
                    pregion(a, nx, nlo, nhi);
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // entry read before the slot refill
                    ptile_issue(nx, nhi, wl32, sl32, lane, a.lane_cap);
                    nstate = 3;
                }
            }
        }
        if (nstate >= 2) {
            cur = nx;
            issued = nstate == 3;
            budget = pipe_quantum_tiles(nbacklog, a.lane_cap);
            if (pstream_region(a, cur, lane)) continue;
            if (lane == 0) {  // nothing left to scan in it
                a.counts[cur.sid] = cur.cnt;
                add_agent(a.queue + kQDone, 1u);
            }
            need_take = true;
            take_t = 0xFFFFFFFFu;
            take_backlog = 0;
            take_claim = 0xFFFFFFFFu;
            continue;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no prefetch may remain in flight
        need_take = true;
        take_t = switching ? tk : 0xFFFFFFFFu;
        take_backlog = nbacklog;
        take_claim = 0xFFFFFFFFu;
    }
}

// ================================================= Rabin-Karp pipelined kernel
// rabinkarp64 (splitter_rabinkarp64.go:26-67, rollinghash Roll):
//   u = v ^ out[leave];  v = (u << 8 | enter) ^ mod[u >> 45]
// Per byte the chain waits on one table read indexed by the hash itself (mod[]), so one
// chain per lane is LDS-latency bound (round 1: 4.07 ms on config 2).  Here each lane runs
// TWO independent chains, A over the first half of its lane segment and B over the second,
// interleaved byte by byte so two mod[] reads are in flight per lane (four per SIMD).
//
// Feeding keeps whole 128-byte lines (64-byte runs cap the DMA at 4.4 vs 6.6 TB/s,
// tools/membench.hip rk): the wave's one 8 KiB step slot receives, per lane, a line of
// chain A and a line of chain B alternately; a chain consumes 64 bytes per step, the
// first half of its line when it arrives and the second half (kept in VGPRs) one step
// later.  A tile (64 lanes x L bytes, L a multiple of 256) is:
//   W     the warm fill [A: 64 B before its half | B: 64 B before its half] (both chains
//         warm from a zero history);
//   2K    line fills (A line 0, B line 0, A line 1, ...), K = L/256 lines per chain;
//   D     drain: B's last 64 bytes (no fill: the slot takes the next tile's warm fill, or
//         the next stream's queue entry).
// (Round 3 tried two bytes per chain hop -- v2 = (v << 16 | c1 c2) ^ T_lo[b] ^ T_hi[a] ^ O16[l1] ^
// outx[l2], GF(2)-linear -- with conflict-free rotated tables: one LDS round trip per two bytes but
// 10.8 VALU per byte instead of 8.9, 2.94-2.97 vs 2.51-2.54 ms on config 2)
// Tables (96 KiB, conflict-free or nearly): out[] with 32 replicas at a 256-byte stride
// (lane l reads replica l % 32, bank pair 2(l % 32); address = one v_perm of the leaving
// byte), mod[] with 16 replicas at a 128-byte stride (lanes l and l+16 share a bank pair
// only for indices of equal parity).  8 waves x 8 KiB slots + 96 KiB = 160 KiB.
//
// Bit-reversed state (round 3).  The hash v (53 bits, deg P = 53) is kept as R = bitreverse64(v)
// in (hi, lo): v's bit j is R's bit 63 - j, so v's low bits -- the ones the cut test reads -- are
// the TOP bits of hi, and `(v & mask) == 0` is `hi < 2^(32 - log2(avg))`: the running test is one
// v_min3 per two bytes instead of a v_and + v_min per byte.  A roll v << 8 | c is R >> 8 with the
// bit-reversed entering byte on top: hi' = one v_perm of hi and the byte (the input dwords are
// bit-reversed once as they leave the step slot, so byte b of w sits bit-reversed in byte 3 - b),
// lo' = one v_alignbit.  The reduction index (v's bits 45..52) is lo's bits 11..18, bit-reversed:
// the tables are stored bit-reversed at bit-reversed rows.  8.9 -> ~7.9 VALU per byte.
// mod[] replicas: 16 = 2-way conflicts and a perm-addressed out[] (32 = conflict-free mod[] but a
// 2-op out[] address: 3.01 vs 2.80 ms on config 2, issue-bound); out[] gets the rest of 96 KiB.
constexpr int kRkModRep = 16;
constexpr int kRkOutRep = 48 - kRkModRep;
struct RkTables {
    uint64_t mod[256 * kRkModRep];  // row f (replicas at f*R + r): rev64(mod[rev8(f)]); first, so its
                                                    // addresses fit the 16-bit ds offset
    uint64_t out[256 * kRkOutRep];  // row f: rev64(outx[rev8(f)]) (outx[] pre-shifted and pre-reduced)
};
static_assert(sizeof(RkTables) + sizeof(RkSlots) <= 160 * 1024, "Rabin-Karp tables + step slots exceed LDS");
constexpr uint32_t kRkIdxBit = 11;  // the reduction index (v >> 45, bit-reversed) = lo bits 11..18

struct RkCtx {
    const char* modb;  // LDS byte address of RkTables::mod
    const char* outb;  // LDS byte address of RkTables::out
    uint32_t lane8o;   // (lane % out replicas) * 8
    uint32_t lane8m;   // (lane % mod replicas) * 8
    uint32_t thr;      // 2^(32 - log2(avg)): a position is a candidate iff hi < thr
};

// The RK kernels' view of a step slot: read_step128, then every dword bit-reversed.
__device__ __forceinline__ void rk_read_step128(const uint8_t* slot, int lane, int64_t c, int64_t off0,
                                                uint32_t (&dw)[32]) {
    read_step128(slot, lane, c, off0, dw);
#pragma unroll
    for (int i = 0; i < 32; i++) dw[i] = __builtin_bitreverse32(dw[i]);
}

// outx[] of the leaving byte b of a (bit-reversed) dword: its row is byte 3 - b.
__device__ __forceinline__ uint64_t rk_out(const RkCtx& k, uint32_t w, int b) {
    const int bb = 3 - b;
    uint32_t a;
    static_assert(kRkOutRep * 8 == 256, "out[]: 256-byte rows, the address in one v_perm");
    a = __builtin_amdgcn_perm(w, k.lane8o, 0x0c0c0000u | ((4u + bb) << 8));  // row << 8 | lane8o
    return *reinterpret_cast<const uint64_t*>(k.outb + a);
}
// v << 8 | c, high word: [hi.b1, hi.b2, hi.b3, the entering byte (byte 3 - b of the reversed dword)]
constexpr uint32_t rk_in_sel(int b) { return 0x00030201u | (static_cast<uint32_t>(7 - b) << 24); }
// mod[] address (16 replicas, 128-byte rows): ((lo >> 4) & 0x7F80) | lane8m as v_lshrrev + one
// v_bitop3 -- both issue every ~2.2-2.4 cycles at two waves per SIMD, where the v_bfe/v_lshl_or or
// v_and_or pairs the compiler picks take ~4.3 each (tools/valu_rate.hip; round 6: the hot loop
// alone 1.728 -> 1.586 ms, tools/rk_loop.hip).
__device__ __forceinline__ uint32_t rk_mod_addr(const RkCtx& k, uint32_t lo) {
    static_assert(kRkModRep == 16, "128-byte mod[] rows");
    return __builtin_amdgcn_bitop3_b32(lo >> (kRkIdxBit - 7), 0xFFu << 7, k.lane8m, 0xEA);  // (x & m) | lane8m
}
// out[] address of the leaving byte b of a (bit-reversed) dword, as rk_out, by one SDWA v_mov that
// writes the byte into byte 1 of `a` and keeps the rest: `a` holds lane8o in byte 0 for good.
__device__ __forceinline__ uint32_t rk_out_sdwa(uint32_t& a, uint32_t w, int b) {
    const int pos = 3 - b;
    if (pos == 0) asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0" : "+v"(a) : "v"(w));
    else if (pos == 1) asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_1" : "+v"(a) : "v"(w));
    else if (pos == 2) asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(a) : "v"(w));
    else asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_3" : "+v"(a) : "v"(w));
    return a;
}
// One roll with the leaving byte's out[] value already read: updates (hi, lo).
// Linearity folds the leaving byte's removal into one table read that is off the chain:
// mod[] is GF(2)-linear in its index and idx(v ^ o) = idx(v) ^ idx(o), so
//   ((v ^ o) << 8 | c) ^ mod[idx(v ^ o)] = ((v << 8) | c) ^ mod[idx(v)] ^ outx[l],
//   outx[l] = (out[l] << 8) ^ mod[idx(out[l])]   (bits 53..60 cancel on both sides).
// The chain is lo -> address (2 VALU) -> mod[] read -> one v_bitop3.
__device__ __forceinline__ void rk_roll(const RkCtx& k, uint32_t& hi, uint32_t& lo, uint64_t ox, uint32_t w, int b) {
    const uint64_t m = *reinterpret_cast<const uint64_t*>(k.modb + rk_mod_addr(k, lo));
    const uint32_t th = __builtin_amdgcn_perm(w, hi, rk_in_sel(b));
    const uint32_t tl = __builtin_amdgcn_alignbit(hi, lo, 8);
    hi = __builtin_amdgcn_bitop3_b32(th, static_cast<uint32_t>(m >> 32), static_cast<uint32_t>(ox >> 32), 0x96);
    lo = __builtin_amdgcn_bitop3_b32(tl, static_cast<uint32_t>(m), static_cast<uint32_t>(ox), 0x96);
}
// Warm roll (leaving byte 0: out[0] = 0).
__device__ __forceinline__ void rk_roll0(const RkCtx& k, uint32_t& hi, uint32_t& lo, uint32_t w, int b) {
    const uint64_t m = *reinterpret_cast<const uint64_t*>(k.modb + rk_mod_addr(k, lo));
    const uint32_t th = __builtin_amdgcn_perm(w, hi, rk_in_sel(b));
    const uint32_t tl = __builtin_amdgcn_alignbit(hi, lo, 8);
    hi = th ^ static_cast<uint32_t>(m >> 32);
    lo = tl ^ static_cast<uint32_t>(m);
}

// 64 bytes of chain A (in a / leaving pa) and of chain B (in b / leaving pb), interleaved
// byte by byte; ma/mb: running min of hi over the piece's positions (a candidate iff < thr).
// Software-pipelined across the chains: a chain's next mod[] read issues right after its own
// roll, so it is in flight while the other chain rolls (one LDS latency + one roll per byte,
// not one latency + two rolls).  The outx[] reads of byte x + W follow each chain's mod[] read
// (the in-order LDS return then never queues a chain's read behind a prefetch).
// ACT_A/ACT_B: whether that chain's bytes are real (an idle chain is not rolled at all).
template <bool ACT_A, bool ACT_B>
__device__ __forceinline__ void rk_step64(const RkCtx& k, uint32_t& ha, uint32_t& la, const uint32_t (&a)[16],
                                          const uint32_t (&pa)[16], uint32_t& hb, uint32_t& lb,
                                          const uint32_t (&b)[16], const uint32_t (&pb)[16], uint32_t& ma,
                                          uint32_t& mb) {
    constexpr int W = 2;  // outx[] reads of both chains issued this many bytes ahead (2: 2.58 ms, 4: 2.65)
    uint64_t oa[64], ob[64];  // only W live at a time (unrolled: register renaming)
    uint32_t xa[W], xb[W];    // out[] address registers (rk_out_sdwa), one per read in flight
#pragma unroll
    for (int i = 0; i < W; i++) xa[i] = xb[i] = k.lane8o;
    auto ld_out = [&](uint32_t& x, uint32_t w, int b) {
        return *reinterpret_cast<const uint64_t*>(k.outb + rk_out_sdwa(x, w, b));
    };
    uint64_t mA = 0, mB = 0;
    if (ACT_A) mA = *reinterpret_cast<const uint64_t*>(k.modb + rk_mod_addr(k, la));
#pragma unroll
    for (int i = 0; i < W; i++)
        if (ACT_A) oa[i] = ld_out(xa[i], pa[i >> 2], i & 3);
    if (ACT_B) mB = *reinterpret_cast<const uint64_t*>(k.modb + rk_mod_addr(k, lb));
#pragma unroll
    for (int i = 0; i < W; i++)
        if (ACT_B) ob[i] = ld_out(xb[i], pb[i >> 2], i & 3);
    uint32_t pha = 0xFFFFFFFFu, phb = 0xFFFFFFFFu;  // the previous byte's hi (tested in pairs)
#pragma unroll
    for (int x = 0; x < 64; x++) {
        __builtin_amdgcn_sched_barrier(0);
        if (ACT_A) {
            const uint32_t th = __builtin_amdgcn_perm(a[x >> 2], ha, rk_in_sel(x & 3));
            const uint32_t tl = __builtin_amdgcn_alignbit(ha, la, 8);
            ha = __builtin_amdgcn_bitop3_b32(th, static_cast<uint32_t>(mA >> 32), static_cast<uint32_t>(oa[x] >> 32), 0x96);
            la = __builtin_amdgcn_bitop3_b32(tl, static_cast<uint32_t>(mA), static_cast<uint32_t>(oa[x]), 0x96);
            __builtin_amdgcn_sched_barrier(0);
            if (x + 1 < 64) mA = *reinterpret_cast<const uint64_t*>(k.modb + rk_mod_addr(k, la));
            if (x + W < 64) oa[x + W] = ld_out(xa[(x + W) % W], pa[(x + W) >> 2], (x + W) & 3);
            __builtin_amdgcn_sched_barrier(0);
            if (x & 1) asm("v_min3_u32 %0, %1, %2, %3" : "=v"(ma) : "v"(ma), "v"(pha), "v"(ha));  // one op per two bytes
            else pha = ha;
        }
        if (ACT_B) {
            const uint32_t th = __builtin_amdgcn_perm(b[x >> 2], hb, rk_in_sel(x & 3));
            const uint32_t tl = __builtin_amdgcn_alignbit(hb, lb, 8);
            hb = __builtin_amdgcn_bitop3_b32(th, static_cast<uint32_t>(mB >> 32), static_cast<uint32_t>(ob[x] >> 32), 0x96);
            lb = __builtin_amdgcn_bitop3_b32(tl, static_cast<uint32_t>(mB), static_cast<uint32_t>(ob[x]), 0x96);
            __builtin_amdgcn_sched_barrier(0);
            if (x + 1 < 64) mB = *reinterpret_cast<const uint64_t*>(k.modb + rk_mod_addr(k, lb));
            if (x + W < 64) ob[x + W] = ld_out(xb[(x + W) % W], pb[(x + W) >> 2], (x + W) & 3);
            __builtin_amdgcn_sched_barrier(0);
            if (x & 1) asm("v_min3_u32 %0, %1, %2, %3" : "=v"(mb) : "v"(mb), "v"(phb), "v"(hb));
            else phb = hb;
        }
    }
}

// Exact re-run of one chain's 64 bytes from (hi, lo) (rare): first index in [lo_i, hi_i]
// that is a candidate, else 64.
__device__ uint32_t rk_exact64(const RkCtx& k, uint32_t hi, uint32_t lo, const uint32_t (&in)[16],
                               const uint32_t (&prv)[16], int lo_i, int hi_i) {
    // 16-byte windows (the arrays shift by four dwords per window, not one per 4 bytes), done
    // once every lane running it has found its candidate
    uint32_t e[16], o[16];
#pragma unroll
    for (int j = 0; j < 16; j++) {
        e[j] = in[j];
        o[j] = prv[j];
    }
    uint32_t first = 64;
#pragma unroll 1
    for (int w = 0; w < 4; w++) {
#pragma unroll
        for (int b = 0; b < 16; b++) {
            rk_roll(k, hi, lo, rk_out(k, o[b >> 2], b & 3), e[b >> 2], b & 3);
            const int i = 16 * w + b;
            if (first == 64 && hi < k.thr && i >= lo_i && i <= hi_i) first = static_cast<uint32_t>(i);
        }
        if (__ballot(first == 64) == 0) break;
#pragma unroll
        for (int q = 0; q < 12; q++) {
            e[q] = e[q + 4];
            o[q] = o[q + 4];
        }
    }
    return first;
}

// Warm fill of a tile -> both chains' 64-byte histories (pa, pb) and states.
__device__ __forceinline__ void rk_warm(const RkCtx& kx, const uint32_t (&dw)[32], uint32_t& ha, uint32_t& la,
                                        uint32_t& hb, uint32_t& lb, uint32_t (&pa)[16], uint32_t (&pb)[16]) {
    ha = la = hb = lb = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) {
        pa[i] = dw[i];
        pb[i] = dw[16 + i];
    }
#pragma unroll
    for (int x = 0; x < 64; x++) {
        if (x % 16 == 0) __builtin_amdgcn_sched_barrier(0);
        rk_roll0(kx, ha, la, pa[x >> 2], x & 3);
        rk_roll0(kx, hb, lb, pb[x >> 2], x & 3);
    }
}
__device__ __forceinline__ RkCtx rk_setup(RkTables& smt, const BatchArgs& a, int lane) {
    auto rev8 = [](uint32_t f) { return __builtin_bitreverse32(f) >> 24; };
    for (uint32_t i = threadIdx.x; i < 256u * kRkModRep; i += blockDim.x)
        smt.mod[i] = __builtin_bitreverse64(a.rk_mod[rev8(i / kRkModRep)]);
    for (uint32_t i = threadIdx.x; i < 256u * kRkOutRep; i += blockDim.x) {  // outx[] (rk_roll)
        const uint64_t o = a.rk_out[rev8(i / kRkOutRep)];
        smt.out[i] = __builtin_bitreverse64((o << 8) ^ a.rk_mod[(o >> 45) & 0xFFu]);
    }
    __syncthreads();
    RkCtx kx;
    kx.modb = reinterpret_cast<const char*>(smt.mod);
    kx.outb = reinterpret_cast<const char*>(smt.out);
    kx.lane8o = static_cast<uint32_t>(lane & (kRkOutRep - 1)) * 8u;
    kx.lane8m = static_cast<uint32_t>(lane & (kRkModRep - 1)) * 8u;
    kx.thr = 1u << (32 - __builtin_popcount(a.mask));  // mask = avg - 1, avg a power of two in [2, 2^31]
    return kx;
}
#define RK_STEP rk_step64
// The rare exact re-run of a 64-byte piece at coordinate c whose running test passed.
__device__ __forceinline__ uint32_t rk_exact(const RkCtx& k, uint32_t h0, uint32_t l0, const Loader& ld, int64_t c,
                                            const uint32_t (&in)[16], const uint32_t (&prv)[16], int lo_i, int hi_i) {
    (void)ld;
    (void)c;
    return rk_exact64(k, h0, l0, in, prv, lo_i, hi_i);
}

// Geometry of a Rabin-Karp tile at ct: L bytes per lane (a multiple of 256: two chains of
// whole 128-byte lines), K lines per chain.
struct RkGeom {
    int64_t L;
    int K;
    Loader ld;
};
__device__ __forceinline__ RkGeom rk_geom(int64_t ct, int64_t hi, const uint8_t* abase, int64_t off0,
                                          int64_t nbytes_coord, int64_t lane_cap = kLaneMax) {
    const int64_t rem = hi - ct + 1;
    int64_t per = (rem + kWave - 1) / kWave;
    per = (per + 255) & ~int64_t(255);
    RkGeom g;
    g.L = per < lane_cap ? per : lane_cap;  // lane_cap: a multiple of 256
    g.K = static_cast<int>(g.L / 256);
    g.ld = make_loader(abase, off0, nbytes_coord, ct >= 64 ? ct - 64 : 0);
    return g;
}
// Warm fill: lane l's slot line = [64 B before c0 | 64 B before c0 + L/2] (16-byte granule j
// of lane l at j ^ sw(l), as dma_step128).
__device__ __forceinline__ void rk_dma_warm(const Loader& ld, uint32_t slot, int64_t ct, int64_t L, int lane) {
    uint32_t sl = slot;  // opaque per call (as dma_step128)
    asm volatile("" : "+s"(sl));
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const int l = 8 * i + (lane >> 3);
        const int jj = (lane & 7) ^ ((l >> 1) & 7);
        const int64_t c0 = ct + l * L + (jj < 4 ? 0 : L / 2);
        const int64_t coord = c0 - 64 + 16 * (jj & 3);
        dma_lds16(ld.d, sl + 1024u * i, static_cast<int32_t>(coord - ld.tb));
    }
}
// Line fill f (1..2K): odd f = line (f-1)/2 of chain A, even f = line f/2 - 1 of chain B.
__device__ __forceinline__ void rk_dma_line(const Loader& ld, uint32_t slot, int64_t ct, int64_t L, int f, int lane) {
    const int64_t half = (f & 1) ? 0 : L / 2;
    const int64_t line = (f & 1) ? (f - 1) / 2 : f / 2 - 1;
    dma_step128(ld, ld.tb, slot, ct + half, L, line, lane);
}
__device__ __forceinline__ void rk_mask_head(uint32_t (&dw)[16], int64_t c, int64_t off0) {
    if (c == 0 && off0) {  // bytes before the stream start are virtual zeros
#pragma unroll
        for (int d = 0; d < 4; d++) {
            const int64_t keep_from = off0 - 4 * d;
            const uint32_t m = keep_from <= 0 ? 0xFFFFFFFFu : (keep_from >= 4 ? 0u : (0xFFFFFFFFu << (8 * keep_from)));
            dw[d] &= m;
        }
    }
}

// The line fills and drain of one tile (after its warm fill, which left both chains' states
// and histories in ha/la, hb/lb, pa, pb): refill(f) is called right after fill f has been
// read out of the slot (the slot is free), check(min, chain, offset from the chain's start,
// state before, bytes, history) after each chain's 64 bytes.  Coordinates stay out of the
// walk (64-bit per-lane values live across it spilled, and every reload's vmcnt wait drained
// the line DMA): `head` says whether lane 0's chain A starts at coordinate 0.
// KCDC_TRACE builds time every line fill's DMA wait (s_memtime, shader cycles) into `dmaw`.
#if KCDC_TRACE
#define RK_VMWAIT(acc)                                                  \
    do {                                                                \
        const uint64_t t0_ = __builtin_amdgcn_s_memtime();              \
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                \
        acc += __builtin_amdgcn_s_memtime() - t0_;                      \
    } while (0)
#else
#define RK_VMWAIT(acc) asm volatile("s_waitcnt vmcnt(0)" ::: "memory")
#endif
template <class Refill, class Check>
__device__ __forceinline__ void rk_walk(const RkCtx& kx, const uint8_t* sl, int lane, bool head,
                                        int64_t off0, int K, uint32_t& ha, uint32_t& la, uint32_t& hb, uint32_t& lb,
                                        uint32_t (&pa)[16], uint32_t (&pb)[16], Refill&& refill, Check&& check,
                                        uint64_t& dmaw) {
    (void)dmaw;
    uint32_t bf[16];  // the second half of the line that arrived last step
#pragma unroll
    for (int i = 0; i < 16; i++) bf[i] = 0;
    for (int j = 0; j < K; j++) {
        // ---- odd fill 2j+1: A line j (A: its first half; B: the second half of its line j-1)
        {
            uint32_t dw[32], na[16];
            __builtin_amdgcn_sched_barrier(0);
            RK_VMWAIT(dmaw);
            rk_read_step128(sl, lane, head && j == 0 ? 0 : 1, off0, dw);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            refill(2 * j + 1);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < 16; i++) na[i] = dw[i];
            const uint32_t ha0 = ha, la0 = la, hb0 = hb, lb0 = lb;
            uint32_t ma = 0xFFFFFFFFu, mb = 0xFFFFFFFFu;
            if (j == 0) {
                RK_STEP<true, false>(kx, ha, la, na, pa, hb, lb, bf, pb, ma, mb);
            } else {
                RK_STEP<true, true>(kx, ha, la, na, pa, hb, lb, bf, pb, ma, mb);
                check(mb, 1, 128 * (j - 1) + 64, hb0, lb0, bf, pb);
#pragma unroll
                for (int i = 0; i < 16; i++) pb[i] = bf[i];
            }
            check(ma, 0, 128 * j, ha0, la0, na, pa);
#pragma unroll
            for (int i = 0; i < 16; i++) {
                pa[i] = na[i];
                bf[i] = dw[16 + i];  // A's second half, next step
            }
        }
        // ---- even fill 2j+2: B line j (A: the second half of its line j; B: its first half)
        {
            uint32_t dw[32], nb[16];
            __builtin_amdgcn_sched_barrier(0);
            RK_VMWAIT(dmaw);
            rk_read_step128(sl, lane, 1, off0, dw);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            refill(2 * j + 2);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < 16; i++) nb[i] = dw[i];
            const uint32_t ha0 = ha, la0 = la, hb0 = hb, lb0 = lb;
            uint32_t ma = 0xFFFFFFFFu, mb = 0xFFFFFFFFu;
            RK_STEP<true, true>(kx, ha, la, bf, pa, hb, lb, nb, pb, ma, mb);
            check(ma, 0, 128 * j + 64, ha0, la0, bf, pa);
            check(mb, 1, 128 * j, hb0, lb0, nb, pb);
#pragma unroll
            for (int i = 0; i < 16; i++) {
                pa[i] = bf[i];
                pb[i] = nb[i];
                bf[i] = dw[16 + i];  // B's second half, next step
            }
        }
    }
    // ---- D: B's last 64 bytes (the slot meanwhile takes the next warm fill / entry)
    {
        const uint32_t hb0 = hb, lb0 = lb;
        uint32_t ma = 0xFFFFFFFFu, mb = 0xFFFFFFFFu;
        RK_STEP<false, true>(kx, ha, la, bf, pa, hb, lb, bf, pb, ma, mb);
        check(mb, 1, 128 * (K - 1) + 64, hb0, lb0, bf, pb);
    }
}

// Rabin-Karp lane segments: twice the buzhash cap (warm-up vs tile overshoot; 2 vs 1: 4M 2.542 vs
// 2.554 ms, 128K 5.536 vs 5.643 ms, profiles/r03/rk/kbench_lmul_*.log)
constexpr int64_t kRkLaneMul = 2;
// Intra-region help as in split_batch_pipe_kernel (the same help slots, claim words and rows; hep,
// hs and the kHs* flags mean the same).  An own tile is T = 64 x rk_cap bytes; a help task scans
// one in two sub-tiles of rk_cap / 2 bytes per lane.
__global__ __launch_bounds__(kRkWaves * kWave, kRkWaves / 4) void split_batch_rk_kernel(BatchArgs a) {
    __shared__ RkTables smt;
    __shared__ RkSlots smslots;
    const int lane = threadIdx.x & (kWave - 1);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const RkCtx kx = rk_setup(smt, a, lane);
    uint8_t* sl = smslots.b[wave][0];
    const uint32_t sl32 = lds_addr(sl);
    const int64_t mx = static_cast<int64_t>(a.max_size);
    const uint32_t me = blockIdx.x * kRkWaves + wave;  // this wave's help slot
    const int64_t rk_cap = kRkLaneMul * static_cast<int64_t>(a.lane_cap);  // lane bytes of an own tile (>= 512)

#if KCDC_TRACE  // per wave at trace[8 * global wave]: start, end, ticks in blocking takes, the last take's
                // start (s_memrealtime); help tiles | own tiles << 32; shader cycles in line-fill DMA
                // waits, in the walks, in the warm fills (s_memtime)
    const uint32_t gw = blockIdx.x * kRkWaves + wave;
    uint64_t tr_block = 0, tr_last = 0, tr_tiles = 0, tr_dma = 0, tr_walk = 0, tr_warm = 0;
    const uint64_t tr_mt0 = __builtin_amdgcn_s_memtime();  // span in shader cycles after the records
    if (lane == 0) a.trace[8 * gw] = __builtin_amdgcn_s_memrealtime();
#define KCDC_RKRET                                                                \
    do {                                                                          \
        if (lane == 0) {                                                          \
            a.trace[8 * gw + 1] = __builtin_amdgcn_s_memrealtime();                \
            a.trace[8 * gw + 2] = tr_block;                                       \
            a.trace[8 * gw + 3] = tr_last;                                        \
            a.trace[8 * gw + 4] = tr_tiles;                                       \
            a.trace[8 * gw + 5] = tr_dma;                                         \
            a.trace[8 * gw + 6] = tr_walk;                                        \
            a.trace[8 * gw + 7] = tr_warm;                                        \
            a.trace[8ull * gridDim.x * kRkWaves + gw] = __builtin_amdgcn_s_memtime() - tr_mt0; \
        }                                                                         \
        return;                                                                   \
    } while (0)
#else
    uint64_t tr_dma = 0;
#define KCDC_RKRET return
#endif
    PStream cur;
    int64_t budget = kNoYield;
    uint32_t hep = 0, hs = 0;
    constexpr uint32_t kHsPub = 1u << 16, kHsNeedPub = 1u << 17, kHsHelped = 1u << 18;
    hs = kHsNeedPub;
    auto hK = [&] { return hs & 0xFFu; };
    auto htile = [&] { return (hs >> 8) & 0xFFu; };
    auto take_blocking = [&](uint32_t t, int64_t backlog_hint, uint32_t claim) -> bool {
#if KCDC_TRACE
        const uint64_t tb0 = __builtin_amdgcn_s_memrealtime();
        tr_last = tb0;
        struct Acc {
            uint64_t t0, &sum;
            __device__ ~Acc() { sum += __builtin_amdgcn_s_memrealtime() - t0; }
        } acc{tb0, tr_block};
#endif
        for (;;) {
            int64_t backlog = backlog_hint;
            if (t == 0xFFFFFFFFu) {
                const uint64_t ht = qht_take(a, lane, 1);
                t = static_cast<uint32_t>(ht);
                backlog = static_cast<int64_t>(ht >> 32) - static_cast<int64_t>(t) - 1;
            }
            const uint32_t held = t;
            const int r = presolve(a, lane, held, cur, kRkWaves, me, a.help != nullptr && claim == 0xFFFFFFFFu);
            if (r == 0) return false;
            if (r == 3) {  // a help task; the ticket stays held (in cap, unused by help tasks, and in memory)
                held_put(a, lane, me, held);
                cur.cap = held;
                uniformize(cur);
                return true;
            }
            t = 0xFFFFFFFFu;
            if (claim != 0xFFFFFFFFu) {
                const bool requeued = bcast(claim) == 2u;
                claim = 0xFFFFFFFFu;
                if (requeued) continue;
            }
            if (r == 2) continue;  // tombstone
            uniformize(cur);
            if (!pcheck(a, lane, cur, held, 1)) return false;
            budget = pipe_quantum(backlog);
            if (pstream_region(a, cur, lane)) return true;
            if (lane == 0) {
                a.counts[cur.sid] = cur.cnt;
                add_agent(a.queue + kQDone, 1u);
            }
        }
    };
    bool need_take = true;
    uint32_t take_t = 0xFFFFFFFFu, take_claim = 0xFFFFFFFFu;
    int64_t take_backlog = 0;
    {
        uint32_t claim = 1u;
        if (lane == 0) {
            claim = 0u;
            __hip_atomic_compare_exchange_strong((gu32*)(a.queue + kQFlags + blockIdx.x), &claim, 1u,
                                                 __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        const uint32_t t0 = first_ticket(blockIdx.x, wave);
        const int64_t nw = static_cast<int64_t>(gridDim.x) * kRkWaves;
        take_t = t0 < a.nstreams ? t0 : 0xFFFFFFFFu;
        take_backlog = static_cast<int64_t>(a.nstreams) - nw;
        take_claim = t0 < a.nstreams ? (claim & 3u) : 0xFFFFFFFFu;
    }
    bool issued = false;  // this tile's warm fill is in flight
    for (;;) {
#if KCDC_HELP_DIAG
        diag_record(a, lane, divergent_bit(need_take, 0) | divergent_bit(take_t, 1) | divergent_bit(issued, 2));
#endif
        if (need_take) {
            if (!take_blocking(take_t, take_backlog, take_claim)) KCDC_RKRET;
            need_take = false;
            issued = false;
            hs |= kHsNeedPub;
        }
#if KCDC_HELP_DIAG
        diag_record(a, lane, divergent_bit(hs, 3) | divergent_bit(hep, 4) | divergent_bit(cur.sid, 5) |
                                 divergent_bit(static_cast<uint32_t>(cur.cap), 6) |
                                 divergent_bit(static_cast<uint32_t>(cur.ct), 7) |
                                 divergent_bit(static_cast<uint32_t>(budget), 8));
#endif
        uniformize(cur);
        if (!pcheck(a, lane, cur, 0xFFFFFFFFu, 5)) KCDC_RKRET;
        const bool is_help = (cur.sid & kHelpBit) != 0;
#if KCDC_TRACE
        tr_tiles += is_help ? 1ull : (1ull << 32);
        const uint64_t tr_t0 = __builtin_amdgcn_s_memtime();
#endif
        int64_t lo, hi;
        pregion(a, cur, lo, hi);
        const int64_t lcap = is_help ? rk_cap / 2 : rk_cap;
        const RkGeom g = rk_geom(cur.ct, hi, cur.abase, cur.off0, cur.off0 + cur.n, lcap);
        const int64_t ct = cur.ct, ct_next = ct + kWave * g.L;
        const bool last_of_region = ct_next > hi;
        // A region new to this wave: publish it when it is long enough to share.
        if ((hs & kHsNeedPub) && !is_help) {
            const int64_t T = kWave * rk_cap;
            const uint32_t K = static_cast<uint32_t>((hi - ct + T) / T);
            hs = 0;
            if (a.help && help_phase(budget) && K >= kHelpMinTiles && K <= static_cast<uint32_t>(kHelpTiles)) {
                const uint32_t Kw = a.help_window && K > a.help_window ? a.help_window : K;  // a window
                hep++;
                hs = kHsPub | Kw;
                help_publish(a, lane, me, hep, cur, ct, Kw < K ? ct + static_cast<int64_t>(Kw) * T - 1 : hi, Kw, T);
            }
        }
        // The owner's claim on its next tile: an atomic add on its slot's bottom after fill 1's
        // DMA, its value consumed at fill 2 (after that fill's vmcnt wait, before its DMA), so
        // no compiler-visible load is in flight across a DMA.
        const bool claim_next_r = (hs & kHsPub) && !is_help && !last_of_region && htile() + 1u < hK();
        const bool budget_out = !is_help && !(hs & kHsHelped) && budget - kWave * g.L <= 0;
        bool ends_nocand = false;
        if (!is_help && last_of_region) {
            const int64_t s2 = cur.s + mx - 1 <= cur.n - 1 ? cur.s + mx : cur.n;
            ends_nocand = s2 >= cur.n || s2 + static_cast<int64_t>(a.min_size) - 1 >= cur.n;
        }
        const bool switching = !is_help && (budget_out || ends_nocand);
        const bool reserve = budget_out && !ends_nocand;
        const bool claim_next = claim_next_r && !switching;
        uint64_t ht_raw = 0;
        if (switching) ht_raw = qht_add(a, lane, 1);  // the next stream's ticket
        uint32_t ht_lo = static_cast<uint32_t>(ht_raw), ht_hi = static_cast<uint32_t>(ht_raw >> 32);
        if (!issued) rk_dma_warm(g.ld, sl32, ct, g.L, lane);
        uint32_t ha = 0, la = 0, hb = 0, lb = 0;
        uint32_t pa[16], pb[16];
        // ---- W: warm fill -> both chains' 64-byte histories; line 1 (A line 0) goes out
        {
            uint32_t dw[32];
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_waitcnt vmcnt(0)" : "+v"(ht_lo), "+v"(ht_hi)::"memory");
            rk_read_step128(sl, lane, -1, cur.off0, dw);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            rk_dma_line(g.ld, sl32, ct, g.L, 1, lane);
            __builtin_amdgcn_sched_barrier(0);
            rk_warm(kx, dw, ha, la, hb, lb, pa, pb);
        }
#if KCDC_TRACE
        const uint64_t tr_t1 = __builtin_amdgcn_s_memtime();
        tr_warm += tr_t1 - tr_t0;
#endif
        uint32_t tk = 0;
        int64_t nbacklog = 0;
        if (switching) {
            const uint64_t ht = qht_value(ht_lo, ht_hi);
            tk = static_cast<uint32_t>(ht);
            nbacklog = static_cast<int64_t>(ht >> 32) + (reserve ? 1 : 0) - static_cast<int64_t>(tk) - 1;
        }
        uint64_t pe_raw = 0;
        bool res_issued = false, next_issued = false, entry_issued = false;
        bool claim_ok = false, claim_known = !claim_next;
        uint64_t claim_raw = 0;
        auto claim_decode = [&]() {  // the claim word before this tile's add (+1 = after it)
            const uint64_t cw = qht_value(static_cast<uint32_t>(claim_raw), static_cast<uint32_t>(claim_raw >> 32)) + 1ull;
            const uint32_t top = static_cast<uint32_t>(cw >> 20) & 0xFFFFFu, bot = static_cast<uint32_t>(cw) & 0xFFFFFu;
            claim_ok = static_cast<uint32_t>(cw >> 40) == hep && bot <= top;
            if (top < hK()) hs |= kHsHelped;
            claim_known = true;
        };
        // After the tile's last fill: the next tile's warm fill, or the next stream's entry.
        auto refill_last = [&]() {
            if (reserve && !res_issued) {  // this stream's ring entry, reserved late
                pe_raw = qht_add(a, lane, 1ull << 32);
                res_issued = true;
            }
            if (switching) {
                pentry_dma(a, lane, tk, sl32);
                entry_issued = true;
            } else if (!last_of_region && (!claim_next || claim_ok)) {  // the next tile has its own geometry
                const RkGeom gn = rk_geom(ct_next, hi, cur.abase, cur.off0, cur.off0 + cur.n, lcap);
                rk_dma_warm(gn.ld, sl32, ct_next, gn.L, lane);
                next_issued = true;
            }
        };
        int32_t found_a = -1, found_b = -1;  // offsets from the chain's start
        // After line fill f is read: issue what the slot takes next (fill f+1, or after the
        // last fill the next tile's warm fill / the next stream's queue entry).
        auto refill = [&](int f) {
            if (claim_next && f == 2) claim_decode();
            if (f < 2 * g.K)
                rk_dma_line(g.ld, sl32, ct, g.L, f + 1, lane);
            else
                refill_last();
            if (claim_next && f == 1 && lane == 0)
                claim_raw = __hip_atomic_fetch_add((gu64*)help_claim(a, me), 1ull, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
        };
        // Hit check of one chain's 64 bytes at `rel` from its start (state before: h0/l0):
        // the chain's first candidate in [lo, hi].  The coordinate is formed only here, from
        // wave-uniform values and an opaque lane id (nothing 64-bit per lane lives across the walk).
        auto check = [&](uint32_t mm, int chain, int rel, uint32_t h0, uint32_t l0, const uint32_t (&in)[16],
                         const uint32_t (&prv)[16]) {
            if (mm < kx.thr && (chain ? found_b : found_a) < 0) {
                int ln = lane;
                asm volatile("" : "+v"(ln));
                const int64_t c = ct + ln * g.L + (chain ? g.L / 2 : 0) + rel;
                if (c <= hi) {
                    const int64_t blo = lo - c, bhi = hi - c;
                    const uint32_t idx = rk_exact(kx, h0, l0, g.ld, c, in, prv, blo < 0 ? 0 : static_cast<int>(blo),
                                                  bhi > 63 ? 63 : static_cast<int>(bhi));
                    if (idx < 64u) {
                        if (chain)
                            found_b = rel + static_cast<int32_t>(idx);
                        else
                            found_a = rel + static_cast<int32_t>(idx);
                    }
                }
            }
        };
        rk_walk(kx, sl, lane, ct == 0 && lane == 0, cur.off0, g.K, ha, la, hb, lb, pa, pb, refill, check, tr_dma);
#if KCDC_TRACE
        tr_walk += __builtin_amdgcn_s_memtime() - tr_t1;
#endif
        const int64_t c0 = ct + lane * g.L;
        const int64_t found = found_a >= 0 ? c0 + found_a : found_b >= 0 ? c0 + g.L / 2 + found_b : -1;
        // ---- end of tile
        if (!claim_known) {  // one-line tiles (K = 1) consume the claim here
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            claim_decode();
        }
        if (reserve && !res_issued) {
            pe_raw = qht_add(a, lane, 1ull << 32);
            res_issued = true;
        }
        const uint64_t hit = __ballot(found >= 0);
        if (is_help) {
            bool done = true;
            if (hit || last_of_region) {  // post the tile's first candidate to its owner's row
                int64_t f = -1;
                if (hit) f = static_cast<int64_t>(uni64(static_cast<uint64_t>(__shfl(found, __builtin_ctzll(hit)))));
                help_post(a, lane, static_cast<uint32_t>(cur.cb), cur.epoch, static_cast<uint32_t>(cur.cnt), cur.s, f);
            } else {  // the next sub-tile (prefetched), unless the owner has closed the region
                const uint64_t w = ld_agent64(help_claim(a, static_cast<uint32_t>(cur.cb)));
                done = static_cast<uint32_t>(qht_value(static_cast<uint32_t>(w), static_cast<uint32_t>(w >> 32)) >> 40) !=
                       cur.epoch;
            }
            if (!done) {
                cur.ct = ct_next;
                issued = next_issued;
                continue;
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the post, or a dropped prefetch
            need_take = true;
            take_t = held_get(a, lane, me, static_cast<uint32_t>(cur.cap));
            take_backlog = 0;
            take_claim = 0xFFFFFFFFu;
            continue;
        }
        bool region_changed = true;
        const int64_t forced = cur.s + mx - 1 <= cur.n - 1 ? cur.s + mx : cur.n;
        int64_t cut = -1;  // this region's cut, once known
        if (hit) {
            const int first = __builtin_ctzll(hit);
            const int64_t f = static_cast<int64_t>(uni64(static_cast<uint64_t>(__shfl(found, first))));
            cut = f - cur.off0 + 1;
        } else if (last_of_region) {  // forced cut at max size (splitter_rabinkarp64.go:60-64) or the end
            cut = forced;
        } else if (claim_next && !claim_ok) {  // the helpers hold the rest of the region
            const int64_t T = kWave * rk_cap;
            const int64_t ct0 = ct - static_cast<int64_t>(htile()) * T;  // the published tile 0
            const int64_t r = help_wait(a, lane, me, hep, htile() + 1u, hK(), ct0);
            const int64_t wend = ct0 + static_cast<int64_t>(hK()) * T;  // past the published window
            if (r >= 0) {
                cut = r - cur.off0 + 1;
            } else if (r == -1 && wend <= hi) {  // no candidate in the window: publish the next one
                cur.ct = wend;
                help_close(a, lane, me, hep);
                hs = kHsNeedPub;
                region_changed = false;
            } else if (r == -1) {
                cut = forced;
            } else {  // a tile still pending: scan on from it, unshared
                cur.ct = ct0 + (-2 - r) * T;
                help_close(a, lane, me, hep);
                hs = 0;
                region_changed = false;
            }
        } else {
            cur.ct = ct_next;
            hs += 1u << 8;  // htile++
            budget -= kWave * g.L;
            region_changed = false;
            if ((hs & kHsPub) && htile() >= hK()) {  // past its published window: the next one
                help_close(a, lane, me, hep);
                hs = kHsNeedPub;
            }
        }
        if (cut >= 0) {
            emit_cut(a, cur, lane, cut);
            cur.s = cut;
            cur.ct = -1;
        }
        if (region_changed) {
            if (hs & kHsPub) help_close(a, lane, me, hep);
            hs = kHsNeedPub;
        }
        const bool live = pstream_region(a, cur, lane);
        if (!live && lane == 0) {
            a.counts[cur.sid] = cur.cnt;
            add_agent(a.queue + kQDone, 1u);
        }
        if (!switching && live) {  // same stream, next tile
            issued = next_issued && !region_changed;
            if (next_issued && region_changed) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // stale prefetch
            continue;
        }
        if (hs & kHsPub) help_close(a, lane, me, hep);  // a yielded region is not ours to share any more
        hs = kHsNeedPub;
        if (reserve) {
            const uint32_t pe = static_cast<uint32_t>(
                qht_value(static_cast<uint32_t>(pe_raw), static_cast<uint32_t>(pe_raw >> 32)) >> 32);
            pwrite(a, lane, pe, cur, !live);
        } else if (live) {  // a candidate kept the stream alive past its predicted last tile
            const uint64_t ht = qht_take(a, lane, 1ull << 32);
            pwrite(a, lane, static_cast<uint32_t>(ht >> 32), cur, false);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the entry DMA (or a stale prefetch) has landed
        bool took = false;
        if (switching && entry_issued) {
            const u32x4 ev = *reinterpret_cast<const u32x4*>(sl + 16 * (lane & 7));
            if (pentry_ok(ev, lane, tk) && static_cast<uint32_t>(__builtin_amdgcn_readlane(ev.w, 0)) != kTombstone) {
                PStream nx;
                pentry_decode(nx, ev);
                uniformize(nx);
                if (!pcheck(a, lane, nx, tk, 2)) KCDC_RKRET;
                cur = nx;
                budget = pipe_quantum(nbacklog);
                took = true;
                issued = false;
                if (!pstream_region(a, cur, lane)) {
                    if (lane == 0) {
                        a.counts[cur.sid] = cur.cnt;
                        add_agent(a.queue + kQDone, 1u);
                    }
                    need_take = true;
                    take_t = 0xFFFFFFFFu;
                    take_backlog = 0;
                    take_claim = 0xFFFFFFFFu;
                }
                continue;
            }
        }
        if (!took) {
            need_take = true;
            take_t = switching ? tk : 0xFFFFFFFFu;
            take_backlog = nbacklog;
            take_claim = 0xFFFFFFFFu;
        }
    }
}

// Before each pipelined launch: zero the queue header (tail := n) and write ring entries
// 0..n-1 = every stream's initial state; later entries get tag 0 (never a valid tag).
// Head starts at min(n, launch waves): every wave's first ticket is preassigned
// (first_ticket: w * grid + b), taken without an atomic (2048 waves hitting one counter at
// launch serialised for ~100 us).  The help slots' claim words start at zero (nothing published).
__global__ void init_ring_kernel(BatchArgs a, uint32_t nslots, uint32_t nwaves, uint32_t spin_cap,
                                 uint32_t steal_spins) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (a.help && i < a.help_waves) *help_claim(a, i) = 0ull;  // help slot i: nothing published
    if (a.help && i < (a.help_waves + 31u) / 32u) help_bits(a)[i] = 0u;
    if (i < kQHeaderBytes / 4)  // (workgroup flags kQFlags.. start at 0: none has started)
        a.queue[i] = i == static_cast<uint32_t>(kQHT) + 1u ? a.nstreams  // tail = n
                   : i == static_cast<uint32_t>(kQHT) ? (nwaves < a.nstreams ? nwaves : a.nstreams)
                   : i == static_cast<uint32_t>(kQCfg) ? spin_cap
                   : i == static_cast<uint32_t>(kQCfg) + 1u ? steal_spins
                                                      : 0u;
    // Every count starts as KCDC_COUNT_FAILED and is overwritten when its stream finishes: a
    // launch that loses a stream (a wave gave up waiting) can never report it as split.
    if (i < a.nstreams) a.counts[i] = ~0ull;
    if (i >= nslots * 8u) return;
    const uint32_t e = i >> 3, g = i & 7u;
    u32x4 v = {0, 0, 0, 0};
    if (e < a.nstreams && g < static_cast<uint32_t>(kPEntryLanes)) {
        const uint64_t p = reinterpret_cast<uint64_t>(a.ptrs[e]);
        const uint64_t cb = a.cut_base[e];
        const uint64_t cend = cut_end_of(a, e);
        const uint64_t w = g == 0 ? 0ull                           // cnt
                         : g == 1 ? (a.starts ? a.starts[e] : 0ull)  // s
                         : g == 2 ? static_cast<uint64_t>(resume_ct(a, e, a.starts ? static_cast<int64_t>(a.starts[e]) : 0,
                                                                     static_cast<int64_t>(a.lens[e]),
                                                                     static_cast<int64_t>(p & 15u)))  // ct (-1: not set up)
                         : g == 3 ? p
                         : g == 4 ? a.lens[e]
                         : g == 5 ? cb
                         : g == 6 ? (cend > cb ? cend - cb : 0ull)
                                  : 0ull;                          // aux 0, epoch 0
        v = pgranule(e + 1u, w, g == 0 ? e : 0u);
    }
    *reinterpret_cast<u32x4*>(reinterpret_cast<uint8_t*>(a.ring) + static_cast<size_t>(e) * kPEntryStride + 16 * g) = v;
}

// Test hook (KCDC_TEST_FORCE_ERROR): mark a finished launch as failed.
__global__ void poison_counts_kernel(BatchArgs a) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < a.nstreams; i += gridDim.x * blockDim.x)
        a.counts[i] = ~0ull;
}

// FIXED-*: cuts every chunk length (splitter_fixed.go:15-26); reads no data.
__global__ void split_fixed_kernel(BatchArgs a) {
    const uint32_t sid = blockIdx.x;
    if (sid >= a.nstreams) return;
    const uint64_t n = a.lens[sid];
    const uint64_t cb = a.cut_base[sid];
    const uint64_t cend = cut_end_of(a, sid);
    const uint64_t cap = cend > cb ? cend - cb : 0;
    const uint64_t L = a.min_size;
    const uint64_t full = n / L;
    const uint64_t cnt = full + (n % L ? 1 : 0);
    for (uint64_t k = threadIdx.x; k < cnt && k < cap; k += blockDim.x) a.cuts[cb + k] = k < full ? (k + 1) * L : n;
    if (threadIdx.x == 0) a.counts[sid] = cnt;
}

// Streaming-handle support: first candidate in [lo, hi] of one aligned buffer.
template <int KIND>
__global__ __launch_bounds__(kWave) void scan_first_kernel(BatchArgs a, const uint8_t* buf, int64_t len, int64_t lo,
                                                            int64_t hi, int64_t* out) {
    __shared__ HashSmem<KIND> sm;
    fill_tables<KIND>(sm, a);
    const int lane = threadIdx.x & (kWave - 1);
    const auto hash = make_hash<KIND>(sm, a, lane);
    const int64_t f = scan_region(hash, buf, 0, len, lo, hi, lane);
    if (lane == 0) out[0] = f;
}

// Grouped streaming handles: one wave per request, request r = first candidate in [lo, hi]
// of the buffer at base + off (256-byte aligned, `len` bytes, 64 bytes of history first).
template <int KIND>
__global__ __launch_bounds__(kWave) void scan_first_batch_kernel(BatchArgs a, const uint8_t* base,
                                                                 const ScanReq* reqs, int64_t* out) {
    __shared__ HashSmem<KIND> sm;
    fill_tables<KIND>(sm, a);
    const int lane = threadIdx.x & (kWave - 1);
    const auto hash = make_hash<KIND>(sm, a, lane);
    const ScanReq& r = reqs[blockIdx.x];
    const uint64_t off = uni64(r.off);
    const int64_t len = static_cast<int64_t>(uni64(static_cast<uint64_t>(r.len)));
    const int64_t lo = static_cast<int64_t>(uni64(static_cast<uint64_t>(r.lo)));
    const int64_t hi = static_cast<int64_t>(uni64(static_cast<uint64_t>(r.hi)));
    const int64_t f = scan_region(hash, base + off, 0, len, lo, hi, lane);
    if (lane == 0) out[blockIdx.x] = f;
}

// Resident scan server for private streaming handles (kcdc_splitter_next): one workgroup
// stays on the GPU while handles are busy and takes requests from a mailbox in fine-grained
// (coherent) host memory, so a NextSplitPoint pays no kernel launch and no table fill.
// Per request: all 512 threads copy the slice (mapped host staging) into device scratch
// with every load in flight, then 8 waves scan 8 sub-ranges of [lo, hi] and the smallest
// first candidate wins.  The kernel exits after kSrvIdle ticks without a request or
// kSrvLife ticks in total (s_memrealtime, 100 MHz); the host relaunches it when needed.
struct ServerMbox {
    uint64_t req_seq;  // host: incremented after the fields below are written
    uint64_t pad0[7];
    uint64_t src;      // device-visible address of the slice (history || bytes)
    int64_t len, lo, hi;
    uint64_t pad1[4];
    uint64_t done_seq;  // device: the request served, after `result`
    int64_t result;
    uint64_t pad2[6];
};
constexpr uint64_t kSrvIdle = 200000;     // 2 ms
constexpr uint64_t kSrvLife = 20000000;   // 200 ms: every server kernel is bounded
constexpr int kSrvWaves = 8;  // 2 per SIMD: scan_region needs up to 219 VGPRs (1,024 threads spilled)

template <int KIND>
__global__ __launch_bounds__(kSrvWaves * kWave) void scan_server_kernel(BatchArgs a, ServerMbox* mb, uint8_t* scratch,
                                                                        uint64_t served) {
    __shared__ HashSmem<KIND> sm;
    __shared__ int64_t wave_first[kSrvWaves];
    __shared__ uint64_t cmd[5];
    fill_tables<KIND>(sm, a);
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    const auto hash0 = make_hash<KIND>(sm, a, lane);
    const uint64_t t0 = wall_clock64();
    uint64_t last = t0;
    for (;;) {
        if (threadIdx.x == 0) {
            uint64_t sq = served;
            for (;;) {
                // relaxed: an acquire at system scope invalidates the L2 on every poll.  The
                // mailbox and the staging are fine-grained host memory (never cached), and the
                // loads below issue only after this loop has exited.
                sq = __hip_atomic_load(&mb->req_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if (sq != served) break;
                const uint64_t now = wall_clock64();
                if (now - last > kSrvIdle || now - t0 > kSrvLife) break;
                __builtin_amdgcn_s_sleep(1);
            }
            cmd[0] = sq;
            if (sq != served) {
                cmd[1] = __hip_atomic_load(&mb->src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                cmd[2] = static_cast<uint64_t>(__hip_atomic_load(&mb->len, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
                cmd[3] = static_cast<uint64_t>(__hip_atomic_load(&mb->lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
                cmd[4] = static_cast<uint64_t>(__hip_atomic_load(&mb->hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
            }
        }
        __syncthreads();
        const uint64_t sq = cmd[0];
        if (sq == served) break;  // idle or lifetime: every thread leaves together
        const uint8_t* src = reinterpret_cast<const uint8_t*>(cmd[1]);
        const int64_t len = static_cast<int64_t>(cmd[2]), lo = static_cast<int64_t>(cmd[3]),
                      hi = static_cast<int64_t>(cmd[4]);
        // the slice -> device scratch (the staging is 256-byte aligned; len <= the scratch).
        // One system-scope acquire per request (not per poll): no line of the staging, which
        // the host rewrites between requests, may be served from a cache.
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
        // 8 loads in flight per thread (64 KiB per round over PCIe), then their stores: a
        // load-store loop left one 16-byte PCIe read per thread outstanding and cost ~2 us per 8 KiB
        const int64_t n16 = len >> 4;
        constexpr int kIn = 8;  // 16-byte PCIe reads in flight per thread while copying a request's slice
        constexpr int64_t kT = kSrvWaves * kWave;
        const u32x4* s16 = reinterpret_cast<const u32x4*>(src);
        u32x4* d16 = reinterpret_cast<u32x4*>(scratch);
        for (int64_t base = 0; base < n16; base += kIn * kT) {
            u32x4 v[kIn];
#pragma unroll
            for (int k = 0; k < kIn; k++) {
                const int64_t i = base + k * kT + threadIdx.x;
                if (i < n16) v[k] = __builtin_nontemporal_load(s16 + i);
            }
#pragma unroll
            for (int k = 0; k < kIn; k++) {
                const int64_t i = base + k * kT + threadIdx.x;
                if (i < n16) d16[i] = v[k];
            }
        }
        for (int64_t i = (n16 << 4) + threadIdx.x; i < len; i += kT) scratch[i] = src[i];
        // Every reader of the scratch is a wave of this workgroup: after the barrier (which waits
        // for the stores) only this CU's vector L1 may still hold the previous request's lines,
        // so invalidate just that (an agent-scope fence would also write back and invalidate
        // the L2 on every request).
        __syncthreads();
        asm volatile("buffer_inv sc0" ::: "memory");
        const int64_t span = hi - lo + 1, per = ((span + kSrvWaves - 1) / kSrvWaves + 63) & ~int64_t(63);
        const int64_t mlo = lo + per * w, mhi = mlo + per - 1 < hi ? mlo + per - 1 : hi;
        int64_t f = -1;
        if (mlo <= mhi) f = scan_region(hash0, scratch, 0, len, mlo, mhi, lane);
        if (lane == 0) wave_first[w] = f;
        __syncthreads();
        if (threadIdx.x == 0) {
            int64_t best = -1;
            for (int k = 0; k < kSrvWaves; k++)
                if (wave_first[k] >= 0 && (best < 0 || wave_first[k] < best)) best = wave_first[k];
            // result, then (after it has completed) the sequence number the host waits for; a
            // release at system scope would write back the whole L2 first
            __hip_atomic_store(&mb->result, best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(&mb->done_seq, sq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        served = sq;
        last = wall_clock64();
        __syncthreads();
    }
}

// Copy-then-scan form of the scans above, one 8-wave workgroup per request: the request's
// bytes (mapped host staging) are copied into device scratch with 8 16-byte PCIe reads in
// flight per thread, then 8 waves scan 8 sub-ranges of [lo, hi].  One wave reading 64 KiB of
// host memory itself was PCIe-latency bound (41 us per private scan, 54 us per group launch).
constexpr int kCpWaves = 8;  // 64 KiB of PCIe reads in flight; 2 waves per SIMD (scan_region <= 235 VGPRs)
template <int KIND>
__device__ __forceinline__ int64_t scan_request_cp(HashSmem<KIND>& sm, const BatchArgs& a, const uint8_t* src,
                                                   uint8_t* scr, int64_t len, int64_t lo, int64_t hi) {
    __shared__ int64_t wf[kCpWaves];
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    constexpr int kIn = 8;
    constexpr int64_t kT = kCpWaves * kWave;
    const int64_t n16 = len >> 4;
    const u32x4* s16 = reinterpret_cast<const u32x4*>(src);
    u32x4* d16 = reinterpret_cast<u32x4*>(scr);
    for (int64_t b = 0; b < n16; b += kIn * kT) {
        u32x4 v[kIn];
#pragma unroll
        for (int k = 0; k < kIn; k++) {
            const int64_t i = b + k * kT + threadIdx.x;
            if (i < n16) v[k] = __builtin_nontemporal_load(s16 + i);
        }
#pragma unroll
        for (int k = 0; k < kIn; k++) {
            const int64_t i = b + k * kT + threadIdx.x;
            if (i < n16) d16[i] = v[k];
        }
    }
    for (int64_t i = (n16 << 4) + threadIdx.x; i < len; i += kT) scr[i] = src[i];
    __syncthreads();
    asm volatile("buffer_inv sc0" ::: "memory");  // this CU's L1 may hold an earlier request's lines
    const auto hash = make_hash<KIND>(sm, a, lane);
    const int64_t span = hi - lo + 1, per = ((span + kCpWaves - 1) / kCpWaves + 63) & ~int64_t(63);
    const int64_t mlo = lo + per * w, mhi = mlo + per - 1 < hi ? mlo + per - 1 : hi;
    const int64_t f = mlo <= mhi ? scan_region(hash, scr, 0, len, mlo, mhi, lane) : -1;
    if (lane == 0) wf[w] = f;
    __syncthreads();
    int64_t best = -1;
    for (int k = 0; k < kCpWaves; k++)
        if (wf[k] >= 0 && (best < 0 || wf[k] < best)) best = wf[k];
    return best;
}

template <int KIND>
__global__ __launch_bounds__(kCpWaves * kWave) void scan_first_cp_kernel(BatchArgs a, const uint8_t* buf, int64_t len,
                                                                         int64_t lo, int64_t hi, int64_t* out,
                                                                         uint8_t* scratch) {
    __shared__ HashSmem<KIND> sm;
    fill_tables<KIND>(sm, a);
    const int64_t f = scan_request_cp<KIND>(sm, a, buf, scratch, len, lo, hi);
    if (threadIdx.x == 0) out[0] = f;
}

template <int KIND>
__global__ __launch_bounds__(kCpWaves * kWave) void scan_first_batch_cp_kernel(BatchArgs a, const uint8_t* base,
                                                                               const ScanReq* reqs, int64_t* out,
                                                                               uint8_t* scratch) {
    __shared__ HashSmem<KIND> sm;
    fill_tables<KIND>(sm, a);
    const ScanReq& r = reqs[blockIdx.x];
    const uint64_t off = uni64(r.off);
    const int64_t len = static_cast<int64_t>(uni64(static_cast<uint64_t>(r.len)));
    const int64_t lo = static_cast<int64_t>(uni64(static_cast<uint64_t>(r.lo)));
    const int64_t hi = static_cast<int64_t>(uni64(static_cast<uint64_t>(r.hi)));
    const int64_t f = scan_request_cp<KIND>(sm, a, base + off, scratch + off, len, lo, hi);
    if (threadIdx.x == 0) out[blockIdx.x] = f;
}

// ------------------------------------------------------ synthetic streams
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void fill_prng_kernel(uint8_t* data, uint64_t stride, uint64_t len, uint32_t nstreams, uint64_t seed,
                                 uint64_t first_sid) {
    const uint64_t words = len >> 3;
    const uint64_t total = words * nstreams;
    const uint64_t step = static_cast<uint64_t>(gridDim.x) * blockDim.x;
    for (uint64_t g = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; g < total; g += step) {
        const uint64_t i = g / words, j = g - i * words;
        const uint64_t key = mix64(seed ^ mix64(first_sid + i + 0x632BE59BD9B4E019ull));
        reinterpret_cast<uint64_t*>(data + i * stride)[j] = mix64(key + (j + 1) * 0x9E3779B97F4A7C15ull);
    }
    if (len & 7) {  // tail bytes of each stream
        for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < nstreams; i += step) {
            const uint64_t key = mix64(seed ^ mix64(first_sid + i + 0x632BE59BD9B4E019ull));
            const uint64_t w = mix64(key + (words + 1) * 0x9E3779B97F4A7C15ull);
            for (uint64_t b = 0; b < (len & 7); b++) data[i * stride + words * 8 + b] = static_cast<uint8_t>(w >> (8 * b));
        }
    }
}

// ------------------------------------------- long single stream (config 3)
// Phase 1: every 128 KiB segment (in coordinates) is scanned by one wave (lane
// l: a 2 KiB sub-range with a 64-byte warm-up), which stores the segment's first
// kSegK candidate positions and whether it had more ("truncated").  Phase 2:
// exclusive prefix sum of the stored counts.  Phase 3: compaction into one
// sorted candidate list.  Phase 4: one wave walks the chunk rule over that list
// from LDS windows; where a truncated (candidate-dense) segment may hide the
// candidate it needs, it rescans that range with the same scan_region() the
// batch kernel uses.  The cut set is therefore exactly the sequential one.
constexpr int64_t kSegBytes = kWave * kLaneMax;  // 128 KiB
constexpr int kSegK = 8;
constexpr uint64_t kTruncBit = 1ull << 63;

// One stream of a long-path launch (several streams share one launch: their segments are
// numbered consecutively, stream j owning global segments [seg0, seg0 + its segment count)).
struct LongStream {
    const uint8_t* abase;
    int64_t off0;
    int64_t n;
    int64_t seg0;
    uint64_t* cuts;
    uint64_t cuts_cap;
    uint64_t* count;
    uint64_t pad;
};
struct LongArgs {
    const LongStream* streams;
    uint32_t nstreams;
    int64_t nseg;        // all streams
    uint32_t* seg_cnt;   // stored count | (truncated << 31)
    uint64_t* seg_cand;  // [nseg][kSegK] positions (relative to the segment's stream)
    uint64_t* seg_off;   // exclusive prefix of stored counts
    uint64_t* list;      // compacted candidates (kTruncBit marks the last stored of a truncated segment)
    uint64_t* total;     // [1] number of list entries
    // parallel resolver (resolve_par_kernel); serial == nullptr: every stream resolves serially
    uint32_t* serial;    // [nstreams] 1: this stream needs the serial resolver
    uint32_t* jump;      // [levels][node_cap] successor tables, node k of stream j at lbeg + 2j + k
    uint32_t* forced;    // [node_cap] non-candidate cuts between a node's cut and its successor's
    uint64_t node_cap;
    uint32_t levels;
};

// The stream owning global segment `seg`: the last j with seg0 <= seg (wave-uniform).
__device__ __forceinline__ uint32_t long_stream_of(const LongArgs& g, int64_t seg) {
    uint32_t lo = 0, hi = g.nstreams - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        const int64_t s0 = static_cast<int64_t>(uni64(static_cast<uint64_t>(g.streams[mid].seg0)));
        if (s0 <= seg) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// Rabin-Karp candidate scan of the long path on split_batch_rk_kernel's tile walk (two
// chains per lane, alternating 128-byte line fills, outx[] folding): one 128 KiB segment per
// tile, persistent grid-stride over the segments of every stream of the launch, the next
// segment's warm fill issued during the drain step.  Records what cand_scan_dma_kernel records.
__global__ __launch_bounds__(kRkWaves * kWave, kRkWaves / 4) void cand_scan_rk_kernel(BatchArgs a, LongArgs g) {
    __shared__ RkTables smt;
    __shared__ RkSlots smslots;
    const int lane = threadIdx.x & (kWave - 1);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const RkCtx kx = rk_setup(smt, a, lane);
    uint8_t* sl = smslots.b[wave][0];
    const uint32_t sl32 = lds_addr(sl);
    const int64_t nw = static_cast<int64_t>(gridDim.x) * kRkWaves;
    struct Seg {
        const uint8_t* abase;
        int64_t off0, n, cs, lo, hi;
    };
    auto seg_of = [&](int64_t seg) {
        const LongStream& S = g.streams[long_stream_of(g, seg)];
        Seg q;
        q.off0 = static_cast<int64_t>(uni64(static_cast<uint64_t>(S.off0)));
        q.n = static_cast<int64_t>(uni64(static_cast<uint64_t>(S.n)));
        q.abase = reinterpret_cast<const uint8_t*>(uni64(reinterpret_cast<uint64_t>(S.abase)));
        q.cs = (seg - static_cast<int64_t>(uni64(static_cast<uint64_t>(S.seg0)))) * kSegBytes;
        q.lo = q.cs > q.off0 ? q.cs : q.off0;
        q.hi = (q.cs + kSegBytes < q.off0 + q.n ? q.cs + kSegBytes : q.off0 + q.n) - 1;
        return q;
    };
    auto issue = [&](const Seg& q) {
        const RkGeom t = rk_geom(q.cs, q.hi, q.abase, q.off0, q.off0 + q.n);
        rk_dma_warm(t.ld, sl32, q.cs, t.L, lane);
    };
    int64_t seg = static_cast<int64_t>(blockIdx.x) * kRkWaves + wave;
    if (seg >= g.nseg) return;
    Seg q = seg_of(seg);
    issue(q);
    for (;;) {
        const int64_t nseg_next = seg + nw;
        const bool has_next = nseg_next < g.nseg;
        Seg qn = q;
        if (has_next) qn = seg_of(nseg_next);
        const RkGeom t = rk_geom(q.cs, q.hi, q.abase, q.off0, q.off0 + q.n);
        uint32_t ha, la, hb, lb, pa[16], pb[16];
        {
            uint32_t dw[32];
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            rk_read_step128(sl, lane, -1, q.off0, dw);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            rk_dma_line(t.ld, sl32, q.cs, t.L, 1, lane);
            __builtin_amdgcn_sched_barrier(0);
            rk_warm(kx, dw, ha, la, hb, lb, pa, pb);
        }
        // candidates per chain, two per register: 16-bit offsets from the chain's start (a lane
        // covers at most 2 KiB of a 128 KiB segment tile); halves state live across the walk
        uint32_t fa[kSegK / 2], fb[kSegK / 2];
#pragma unroll
        for (int k = 0; k < kSegK / 2; k++) fa[k] = fb[k] = 0;
        int na = 0, nb = 0;  // candidates per chain (kSegK + 1: more than kSegK)
        auto refill = [&](int f) {
            if (f < 2 * t.K)
                rk_dma_line(t.ld, sl32, q.cs, t.L, f + 1, lane);
            else if (has_next)
                issue(qn);
        };
        auto check = [&](uint32_t mm, int chain, int crel, uint32_t h0, uint32_t l0, const uint32_t (&in)[16],
                         const uint32_t (&prv)[16]) {
            int& nf = chain ? nb : na;
            uint32_t(&fnd)[kSegK / 2] = chain ? fb : fa;
            if (mm < kx.thr && nf <= kSegK) {  // rare: enumerate the piece's candidates exactly
                int ln = lane;
                asm volatile("" : "+v"(ln));  // the coordinate is formed here only (rk_walk)
                const int64_t c = q.cs + ln * t.L + (chain ? t.L / 2 : 0) + crel;
                const int64_t blo = q.lo - c, bhi = q.hi - c;
                int from = blo < 0 ? 0 : static_cast<int>(blo);
                const int to = bhi > 63 ? 63 : static_cast<int>(bhi);
                while (from <= to && nf <= kSegK) {
                    const uint32_t idx = rk_exact(kx, h0, l0, t.ld, c, in, prv, from, to);
                    if (idx >= 64u) break;
                    const uint32_t rel = static_cast<uint32_t>(crel) + idx;  // < 2^16
#pragma unroll
                    for (int k = 0; k < kSegK; k++)  // entry nf = rel, kept in registers (no scratch)
                        if (k == nf) fnd[k >> 1] |= rel << (16 * (k & 1));
                    nf++;
                    from = static_cast<int>(idx) + 1;
                }
            }
        };
        uint64_t dmaw = 0;
        rk_walk(kx, sl, lane, q.cs == 0 && lane == 0, q.off0, t.K, ha, la, hb, lb, pa, pb, refill, check, dmaw);
        const int64_t c0 = q.cs + lane * t.L, c0b = c0 + t.L / 2;
        // this lane's candidates in position order: chain A's, then chain B's
        const int nas = na < kSegK ? na : kSegK;
        const int nf = na + nb > kSegK ? kSegK + 1 : na + nb;
        uint32_t found[kSegK];  // offsets from the segment start
        const uint32_t base_a = static_cast<uint32_t>(c0 - q.cs), base_b = static_cast<uint32_t>(c0b - q.cs);
#pragma unroll
        for (int j = 0; j < kSegK; j++) {
            uint32_t v = base_a + ((fa[j >> 1] >> (16 * (j & 1))) & 0xFFFFu);
#pragma unroll
            for (int k = 0; k < kSegK; k++)
                if (j >= nas && k == j - nas) v = base_b + ((fb[k >> 1] >> (16 * (k & 1))) & 0xFFFFu);
            found[j] = v;
        }
        int incl = nf;
#pragma unroll
        for (int d = 1; d < kWave; d <<= 1) {
            const int v = __shfl_up(incl, d);
            if (lane >= d) incl += v;
        }
        const int tot = __shfl(incl, kWave - 1);
        const int pre = incl - nf;
        for (int j = 0; j < nf && j < kSegK; j++)
            if (pre + j < kSegK) g.seg_cand[seg * kSegK + pre + j] = static_cast<uint64_t>(q.cs - q.off0) + found[j];
        if (lane == 0)
            g.seg_cnt[seg] = (tot > kSegK ? 0x80000000u : 0u) | static_cast<uint32_t>(tot < kSegK ? tot : kSegK);
        if (!has_next) break;
        seg = nseg_next;
        q = qn;
    }
}

// Buzhash candidate scan of the long path on the batch kernel's feeding scheme: a segment
// (128 KiB of coordinates) is exactly one tile of 64 lane segments, streamed by LDS-DMA in
// 128-byte steps with the next segment's warm piece and first step prefetched during the
// last step; persistent grid (one workgroup of kDmaWaves waves per CU), grid-stride over
// the segments of every stream of the launch.  Per segment it records the first kSegK
// candidates (positions from the stream start) and a truncation flag.
template <bool TOP>
__global__ __launch_bounds__(kDmaWaves * kWave, kDmaWaves / 4) void cand_scan_dma_kernel(BatchArgs a, LongArgs g) {
    __shared__ BuzShared smtab;
    __shared__ DmaSlots smslots;
    __shared__ WarmSlots smwarm;
    fill_buz_table(smtab, a.buz, a.buz_rot);
    __syncthreads();
    const int lane = threadIdx.x & (kWave - 1);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    BuzRing hash;
    hash.tab = reinterpret_cast<const char*>(smtab.tab);
    hash.lane4 = static_cast<uint32_t>(lane) * 4u;
    hash.mask = a.mask;
    hash.h = 0;
    uint8_t* sl = smslots.b[wave][0];
    uint8_t* wl = smwarm.b[wave];
    const uint32_t sl32 = lds_addr(sl), wl32 = lds_addr(wl);
    const uint32_t lim = TOP ? a.buz_lim : 0u;
    const int64_t nw = static_cast<int64_t>(gridDim.x) * kDmaWaves;
    struct Seg {
        const uint8_t* abase;
        int64_t off0, n, cs, lo, hi;
    };
    auto seg_of = [&](int64_t seg) {
        const LongStream& S = g.streams[long_stream_of(g, seg)];
        Seg q;
        q.off0 = static_cast<int64_t>(uni64(static_cast<uint64_t>(S.off0)));
        q.n = static_cast<int64_t>(uni64(static_cast<uint64_t>(S.n)));
        q.abase = reinterpret_cast<const uint8_t*>(uni64(reinterpret_cast<uint64_t>(S.abase)));
        q.cs = (seg - static_cast<int64_t>(uni64(static_cast<uint64_t>(S.seg0)))) * kSegBytes;
        q.lo = q.cs > q.off0 ? q.cs : q.off0;
        q.hi = (q.cs + kSegBytes < q.off0 + q.n ? q.cs + kSegBytes : q.off0 + q.n) - 1;
        return q;
    };
    auto issue = [&](const Seg& q) {
        const TileGeom t = tile_geom(q.cs, q.hi, q.abase, q.off0, q.off0 + q.n);
        dma_piece(t.ld, t.ld.tb, wl32, q.cs, t.L, -1, lane);
        dma_step128(t.ld, t.ld.tb, sl32, q.cs, t.L, 0, lane);
    };
    int64_t seg = static_cast<int64_t>(blockIdx.x) * kDmaWaves + wave;
    if (seg >= g.nseg) return;
    Seg q = seg_of(seg);
    issue(q);
    for (;;) {
        const int64_t nseg_next = seg + nw;
        const bool has_next = nseg_next < g.nseg;
        Seg qn = q;
        if (has_next) qn = seg_of(nseg_next);
        const TileGeom t = tile_geom(q.cs, q.hi, q.abase, q.off0, q.off0 + q.n);
        const int64_t c0 = q.cs + lane * t.L;
        {
            uint32_t w16[16];
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            read_piece(wl, lane, c0 - 64, q.off0, w16);
            hash.clear();
            hash.template block<kWarm>(w16);
        }
        uint32_t found[kSegK];
        int nf = 0;  // candidates of this lane (kSegK + 1: more than kSegK)
        for (int nb = 0; nb < t.nb; nb++) {
            const int64_t c = c0 + 128 * nb;
            const typename BuzRing::State st0 = hash.save();
            uint32_t dw[32];
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            read_step128(sl, lane, c, q.off0, dw);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot free: refill it
            __builtin_amdgcn_sched_barrier(0);
            if (nb + 1 < t.nb)
                dma_step128(t.ld, t.ld.tb, sl32, q.cs, t.L, nb + 1, lane);
            else if (has_next)
                issue(qn);
            __builtin_amdgcn_sched_barrier(0);
            const uint32_t m = hash.template step128<TOP>(dw, 0u);
            __builtin_amdgcn_sched_barrier(0);
            if (m <= lim && c <= q.hi && nf <= kSegK) {  // rare: exact re-run from global memory
                uint32_t prv[16], cur32[32];
                t.ld.load(c - 64, prv);
                t.ld.load(c, cur32);
                const int64_t blo = q.lo - c, bhi = q.hi - c;
                int from = blo < 0 ? 0 : static_cast<int>(blo);
                const int to = bhi > 127 ? 127 : static_cast<int>(bhi);
                while (from <= to && nf <= kSegK) {
                    const uint32_t idx = hash.exact(st0, prv, cur32, from, to);
                    if (idx >= 128u) break;
                    if (nf < kSegK) found[nf] = static_cast<uint32_t>(c - q.cs) + idx;
                    nf++;
                    from = static_cast<int>(idx) + 1;
                }
                __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), visible to the waitcnt pass
            }
        }
        // exclusive prefix of per-lane counts (lane segments are in position order)
        int incl = nf;
#pragma unroll
        for (int d = 1; d < kWave; d <<= 1) {
            const int v = __shfl_up(incl, d);
            if (lane >= d) incl += v;
        }
        const int tot = __shfl(incl, kWave - 1);
        const int pre = incl - nf;
        for (int j = 0; j < nf && j < kSegK; j++)
            if (pre + j < kSegK) g.seg_cand[seg * kSegK + pre + j] = static_cast<uint64_t>(q.cs - q.off0) + found[j];
        if (lane == 0)
            g.seg_cnt[seg] = (tot > kSegK ? 0x80000000u : 0u) | static_cast<uint32_t>(tot < kSegK ? tot : kSegK);
        if (!has_next) break;
        seg = nseg_next;
        q = qn;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Exclusive prefix sum of the stored counts over all segments, in three launches:
// per-block sums of kPrefixItems segments, a scan of the block sums (one thread: a few
// hundred blocks at most), then every block scans its items from its offset.
constexpr int kPrefixItems = 1024 * 8;
__global__ __launch_bounds__(1024) void seg_blocksum_kernel(LongArgs g, uint64_t* block_sum) {
    __shared__ uint32_t wsum[16];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int64_t base = static_cast<int64_t>(blockIdx.x) * kPrefixItems;
    uint32_t sum = 0;
    for (int j = 0; j < 8; j++) {
        const int64_t i = base + static_cast<int64_t>(t) * 8 + j;
        sum += i < g.nseg ? (g.seg_cnt[i] & 0x7FFFFFFFu) : 0u;
    }
    for (int d = 32; d >= 1; d >>= 1) sum += __shfl_down(sum, d);
    if (lane == 0) wsum[w] = sum;
    __syncthreads();
    if (t == 0) {
        uint64_t tot = 0;
        for (int k = 0; k < 16; k++) tot += wsum[k];
        block_sum[blockIdx.x] = tot;
    }
}

__global__ void block_offsets_kernel(LongArgs g, uint64_t* block_sum, uint32_t nblocks) {
    if (threadIdx.x != 0) return;
    uint64_t run = 0;
    for (uint32_t b = 0; b < nblocks; b++) {  // in place: block_sum[b] becomes its exclusive offset
        const uint64_t v = block_sum[b];
        block_sum[b] = run;
        run += v;
    }
    g.total[0] = run;
}

__global__ __launch_bounds__(1024) void seg_prefix_kernel(LongArgs g, const uint64_t* block_off) {
    __shared__ uint64_t wsum[16];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    constexpr int kItems = 8;
    const int64_t base = static_cast<int64_t>(blockIdx.x) * kPrefixItems;
    uint32_t v[kItems];
    uint32_t sum = 0;
#pragma unroll
    for (int j = 0; j < kItems; j++) {
        const int64_t i = base + static_cast<int64_t>(t) * kItems + j;
        v[j] = i < g.nseg ? (g.seg_cnt[i] & 0x7FFFFFFFu) : 0u;
        sum += v[j];
    }
    uint32_t incl = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t x = __shfl_up(incl, d);
        if (lane >= d) incl += x;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint64_t run = block_off[blockIdx.x];
    for (int k = 0; k < w; k++) run += wsum[k];
    run += incl - sum;
#pragma unroll
    for (int j = 0; j < kItems; j++) {
        const int64_t i = base + static_cast<int64_t>(t) * kItems + j;
        if (i < g.nseg) g.seg_off[i] = run;
        run += v[j];
    }
}

__global__ void compact_kernel(LongArgs g) {
    const int64_t seg = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (seg >= g.nseg) return;
    const uint32_t c = g.seg_cnt[seg];
    const uint32_t k = c & 0x7FFFFFFFu;
    const uint64_t o = g.seg_off[seg];
    for (uint32_t j = 0; j < k; j++) {
        uint64_t v = g.seg_cand[seg * kSegK + j];
        if ((c >> 31) && j + 1 == k) v |= kTruncBit;
        g.list[o + j] = v;
    }
}

constexpr int kResolveWin = 4096;  // candidate-list entries staged in LDS

// One wave per stream (blockIdx.x): walks the chunk rule over the stream's candidate list.
template <int KIND>
__global__ __launch_bounds__(kWave) void resolve_kernel(BatchArgs a, LongArgs g, int64_t mn, int64_t mx) {
    if (g.serial && g.serial[blockIdx.x] == 0) return;  // resolved by resolve_par_kernel
    __shared__ HashSmem<KIND> sm;
    __shared__ uint64_t win[kResolveWin];
    fill_tables<KIND>(sm, a);
    const int lane = threadIdx.x;
    const auto hash = make_hash<KIND>(sm, a, lane);
    const LongStream& S = g.streams[blockIdx.x];
    const int64_t n = static_cast<int64_t>(uni64(static_cast<uint64_t>(S.n)));
    const int64_t off0 = static_cast<int64_t>(uni64(static_cast<uint64_t>(S.off0)));
    const uint8_t* abase = reinterpret_cast<const uint8_t*>(uni64(reinterpret_cast<uint64_t>(S.abase)));
    const int64_t seg0 = static_cast<int64_t>(uni64(static_cast<uint64_t>(S.seg0)));
    const uint64_t cuts_cap = uni64(S.cuts_cap);
    uint64_t* const cuts = reinterpret_cast<uint64_t*>(uni64(reinterpret_cast<uint64_t>(S.cuts)));
    // this stream's slice of the compacted list
    const int64_t lbeg = seg0 < g.nseg ? static_cast<int64_t>(uni64(g.seg_off[seg0])) : 0;
    const int64_t lend = blockIdx.x + 1 < g.nstreams && uni64(static_cast<uint64_t>(g.streams[blockIdx.x + 1].seg0)) <
                                                            static_cast<uint64_t>(g.nseg)
                             ? static_cast<int64_t>(uni64(g.seg_off[g.streams[blockIdx.x + 1].seg0]))
                             : static_cast<int64_t>(uni64(g.total[0]));
    const uint64_t* const list = g.list + lbeg;
    const int64_t total = n > 0 ? lend - lbeg : 0;
    int64_t wbase = 0;  // list index of win[0]
    auto load_win = [&](int64_t at) {
        __syncthreads();
        for (int j = lane; j < kResolveWin; j += kWave) win[j] = at + j < total ? list[at + j] : ~0ull >> 1;
        __syncthreads();
        wbase = at;
    };
    auto entry = [&](int64_t i) -> uint64_t {  // wave-uniform
        if (i < wbase || i >= wbase + kResolveWin) load_win(i > 64 ? i - 64 : 0);
        return win[i - wbase];
    };
    load_win(0);
    int64_t s = 0, i = 0;
    uint64_t cnt = 0;
    while (s < n) {
        const int64_t lo = s + mn - 1;
        int64_t next;
        if (lo >= n) {
            next = n;
        } else {
            const int64_t hi = s + mx - 1 < n - 1 ? s + mx - 1 : n - 1;
            // advance i to the first entry >= lo, 64 entries per step
            for (;;) {
                if (i >= total) break;
                if (i < wbase || i + kWave > wbase + kResolveWin) load_win(i > 64 ? i - 64 : 0);
                const int64_t j = i + lane;
                const bool ge = j >= total || static_cast<int64_t>(win[j - wbase] & ~kTruncBit) >= lo;
                const uint64_t bal = __ballot(ge);
                if (bal) {
                    i += __builtin_ctzll(bal);
                    break;
                }
                i += kWave;
            }
            if (i > total) i = total;
            int64_t c = -1;
            if (i > 0) {
                const uint64_t e = entry(i - 1);
                if (e & kTruncBit) {  // its segment may hold unlisted candidates >= lo
                    // end (exclusive, in positions) of the coordinate segment holding entry e
                    const int64_t seg_end =
                        ((static_cast<int64_t>(e & ~kTruncBit) + off0) / kSegBytes + 1) * kSegBytes - off0;
                    if (seg_end > lo) {
                        const int64_t rh = seg_end - 1 < hi ? seg_end - 1 : hi;
                        const int64_t f = scan_region(hash, abase, off0, off0 + n, lo + off0, rh + off0, lane);
                        if (f >= 0) c = f - off0;
                    }
                }
            }
            if (c < 0 && i < total) {
                const int64_t p = static_cast<int64_t>(entry(i) & ~kTruncBit);
                if (p <= hi) c = p;
            }
            if (c >= 0)
                next = c + 1;
            else if (s + mx - 1 <= n - 1)
                next = s + mx;
            else
                next = n;
        }
        if (lane == 0 && cnt < cuts_cap) cuts[cnt] = static_cast<uint64_t>(next);
        cnt++;
        s = next;
    }
    if (lane == 0) S.count[0] = cnt;
}

// Parallel chunk resolution of one stream per workgroup (1024 threads), for streams whose
// candidate list is complete (no truncated segment) and fits the node tables.  Nodes: the
// list entries 0..M-1 ("a chunk ends after p_k"), START = M (the stream start) and END.
//  A. succ(k): the node whose candidate ends the chunk after node k's cut, walking the
//     chunk rule from s = p_k + 1 (forced cuts at max size / the stream end in between are
//     counted in forced[k]; they are arithmetic in s).  Candidates are sorted: binary search.
//  B. jump tables: jump_t(k) = succ^(2^t)(k).
//  C. the chain START -> ... -> END: node d of the chain by binary lifting on d, its cut
//     index by a block prefix sum of (1 + forced), then every node writes its own cuts.
// The cut list equals the serial walk's (resolve_kernel) cut for cut.
__device__ __forceinline__ uint32_t lower_bound_pos(const uint64_t* list, uint32_t m, int64_t v) {
    uint32_t lo = 0, hi = m;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (static_cast<int64_t>(list[mid]) < v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(1024) void resolve_par_kernel(LongArgs g, int64_t mn, int64_t mx) {
    __shared__ uint32_t s_flag;
    __shared__ uint64_t s_wsum[16];
    __shared__ uint64_t s_carry;
    __shared__ uint64_t s_depth;
    const uint32_t j = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const LongStream& S = g.streams[j];
    const int64_t n = S.n;
    const int64_t seg0 = S.seg0;
    const int64_t lbeg = seg0 < g.nseg ? static_cast<int64_t>(g.seg_off[seg0]) : 0;
    const int64_t lend = j + 1 < g.nstreams && static_cast<uint64_t>(g.streams[j + 1].seg0) < static_cast<uint64_t>(g.nseg)
                             ? static_cast<int64_t>(g.seg_off[g.streams[j + 1].seg0])
                             : static_cast<int64_t>(g.total[0]);
    const uint32_t M = n > 0 ? static_cast<uint32_t>(lend - lbeg) : 0u;
    const uint64_t nb = static_cast<uint64_t>(lbeg) + 2ull * j;  // this stream's node base
    const uint64_t* list = g.list + lbeg;
    if (tid == 0) s_flag = nb + M + 2 > g.node_cap ? 1u : 0u;
    __syncthreads();
    for (uint32_t k = tid; k < M && !s_flag; k += 1024)
        if (list[k] & kTruncBit) s_flag = 1u;  // benign race: any writer stores 1
    __syncthreads();
    if (s_flag) {
        if (tid == 0) g.serial[j] = 1u;
        return;
    }
    if (tid == 0) g.serial[j] = 0u;
    const uint32_t START = M, END = M + 1;
    uint32_t* J0 = g.jump + nb;
    uint32_t* F = g.forced + nb;
    for (uint32_t k = tid; k <= END; k += 1024) {  // A
        uint32_t sc = END, f = 0;
        if (k != END) {
            int64_t s = k == START ? 0 : static_cast<int64_t>(list[k]) + 1;
            while (s < n) {
                const int64_t lo = s + mn - 1;
                if (lo >= n) {  // the last chunk [s, n)
                    f++;
                    break;
                }
                const int64_t hi = s + mx - 1 < n - 1 ? s + mx - 1 : n - 1;
                const uint32_t q = lower_bound_pos(list, M, lo);
                if (q < M && static_cast<int64_t>(list[q]) <= hi) {
                    sc = q;
                    break;
                }
                f++;  // forced cut at s + mx, or at the stream end
                if (s + mx - 1 <= n - 1) s += mx;
                else break;
            }
        }
        J0[k] = sc;
        F[k] = f;
    }
    __syncthreads();
    const uint64_t stride = g.node_cap;
    for (uint32_t t = 1; t < g.levels; t++) {  // B
        const uint32_t* Jp = g.jump + (t - 1) * stride + nb;
        uint32_t* Jt = g.jump + t * stride + nb;
        for (uint32_t k = tid; k <= END; k += 1024) Jt[k] = Jp[Jp[k]];
        __syncthreads();
    }
    if (tid == 0) {  // chain length: START's depth (number of candidate nodes on the chain)
        uint32_t cur = START;
        uint64_t d = 0;
        for (int t = static_cast<int>(g.levels) - 1; t >= 0; t--) {
            const uint32_t nx = g.jump[static_cast<uint64_t>(t) * stride + nb + cur];
            if (nx != END) {
                cur = nx;
                d += 1ull << t;
            }
        }
        s_depth = d;
        s_carry = 0;
    }
    __syncthreads();
    const uint64_t D = s_depth;  // chain nodes d = 0 (START) .. D
    uint64_t* const cuts = S.cuts;
    const uint64_t cap = S.cuts_cap;
    for (uint64_t base = 0; base <= D; base += 1024) {  // C
        const uint64_t d = base + static_cast<uint64_t>(tid);
        const bool valid = d <= D;
        uint32_t node = START;
        if (valid)
            for (uint32_t t = 0; t < g.levels; t++)
                if ((d >> t) & 1) node = g.jump[static_cast<uint64_t>(t) * stride + nb + node];
        const uint64_t wgt = valid ? F[node] + (d > 0 ? 1u : 0u) : 0u;
        uint64_t incl = wgt;
        for (int o = 1; o < 64; o <<= 1) {
            const uint64_t v = __shfl_up(incl, o);
            if (lane >= o) incl += v;
        }
        if (lane == 63) s_wsum[w] = incl;
        __syncthreads();
        uint64_t pre = s_carry;
        for (int k = 0; k < w; k++) pre += s_wsum[k];
        uint64_t idx = pre + incl - wgt;
        if (valid) {
            int64_t s = 0;
            if (d > 0) {
                s = static_cast<int64_t>(list[node]) + 1;
                if (idx < cap) cuts[idx] = static_cast<uint64_t>(s);
                idx++;
            }
            for (uint32_t r = 0; r < F[node]; r++) {
                const int64_t next = s + mn - 1 >= n ? n : (s + mx - 1 <= n - 1 ? s + mx : n);
                if (idx < cap) cuts[idx] = static_cast<uint64_t>(next);
                idx++;
                s = next;
            }
        }
        __syncthreads();
        if (tid == 1023) {
            uint64_t tot = s_carry;
            for (int k = 0; k < 16; k++) tot += s_wsum[k];
            s_carry = tot;
        }
        __syncthreads();
    }
    if (tid == 0) S.count[0] = s_carry;
}

// Test support (kcdc_test_occupy): hold `nwg` CUs -- one workgroup each, all of the CU's
// LDS -- for `us` microseconds of the 100 MHz constant clock, then exit (bounded).
__global__ __launch_bounds__(64) void occupy_kernel(uint64_t ticks, uint32_t* sink) {
    extern __shared__ uint32_t hold[];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t x = threadIdx.x;
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
        __builtin_amdgcn_s_sleep(127);
        x = x * 1664525u + 1013904223u;
    }
    hold[threadIdx.x] = x;
    __syncthreads();
    if (hold[(threadIdx.x + 1) & 63] == 0x12345678u) sink[0] = x;  // keeps the loop and the LDS live
}

}  // namespace dev

// ================================================================== host
struct DeviceTables {
    uint32_t* buz = nullptr;
    uint64_t* rk_out = nullptr;
    uint64_t* rk_mod = nullptr;
    int cus = 0;
};

namespace {
constexpr int kMaxDevices = 64;
constexpr int kQueueSlots = 64;  // per-launch queue workspaces, chosen round-robin per launch
DeviceTables g_dev_tables[kMaxDevices];
// Queue workspace of one launch slot: header (256 B: head, tail, done, error words 64 B
// apart) | ring (P x 8 B, P = pow2 > nstreams + grid waves) | progress (nstreams x 24 B).
// Grow-only; a replaced buffer is freed once the slot's last launch (its `done` event) finished.
struct QueueWs {
    char* base = nullptr;
    size_t bytes = 0;
    hipEvent_t done = nullptr;  // recorded after the slot's last launch: a reuse from another
                                // stream waits for it (more than kQueueSlots launches in flight)
    hipStream_t last = nullptr;  // the stream of the slot's last launch
    bool used = false;
};
QueueWs g_qws[kMaxDevices][kQueueSlots];
// Slot affinity: back-to-back launches on one stream reuse that stream's slot (stream order
// already serialises them, so no event wait, and the workspace stays warm); other streams
// take slots round-robin.  A few recent streams per device, least recently used replaced.
struct StreamSlot {
    hipStream_t st = nullptr;
    unsigned slot = 0;
    uint64_t tick = 0;
    bool valid = false;
};
constexpr int kStreamSlots = 8;
StreamSlot g_stream_slot[kMaxDevices][kStreamSlots];
uint64_t g_slot_tick[kMaxDevices];
bool g_dev_ready[kMaxDevices];
unsigned g_queue_next[kMaxDevices];
// Per-device locks: table setup and a launch's slot / workspace / enqueue sequence are
// serialised per device only, so threads driving different devices never wait on each other.
std::mutex g_dev_mu[kMaxDevices];

int hip_fail(hipError_t e, const char* what) { return set_error(-5, std::string(what) + ": " + hipGetErrorString(e)); }

// Test hooks (kcdc_test_set, include/kcdc.h "testing"): read by every later launch.
struct TestKnobs {
    uint32_t spin_cap = 0;     // 0: dev::kSpinCap
    bool no_steal = false;     // disable try_steal
    bool force_error = false;  // mark every pipelined launch as failed
    int help = 0;              // intra-region help: 0 the policy below, 1 off, 2 on (A/B, tests)
    uint32_t lane_cap = 0;     // buzhash batch lane segment cap (256..4096, a power of two); 0: base_args' rule
    uint32_t help_window = 0;  // buzhash help window in tiles (255: whole regions); 0: launch_split_batch's rule
    char* last_ws = nullptr;   // queue header of the last pipelined launch (kcdc_test_queue_stat)
    int last_dev = 0;
    uint32_t last_waves = 0;   // launch waves of that launch (kcdc_test_queue_stat key 12)
};
TestKnobs g_test;

// Rotated buzhash frame for a reference mask (avg - 1).  A contiguous low mask of k bits
// (avg a power of two, the registered splitters) rotates to the top k bits: rot = 32 - k,
// and h & mask == 0 <=> h <= ~mask.  Any other mask keeps rot = 0 (top = false).
struct BuzFrame {
    uint32_t rot, mask, lim;
    bool top;
};
BuzFrame buz_frame(uint32_t mask) {
    BuzFrame f{0, mask, 0, false};
    if ((mask & (mask + 1u)) == 0) {  // 0b0..01..1 (including 0 and all ones)
        const uint32_t k = static_cast<uint32_t>(__builtin_popcount(mask));
        f.rot = (32u - k) & 31u;
        f.mask = f.rot ? (mask << f.rot) | (mask >> (32u - f.rot)) : mask;
        f.lim = ~f.mask;
        f.top = true;
    }
    return f;
}

dev::BatchArgs base_args(const Algo& algo, const DeviceTables& t) {
    dev::BatchArgs a{};
    a.min_size = algo.min_size();
    a.max_size = algo.max_size();
    a.mask = static_cast<uint32_t>(algo.mask());
    if (algo.kind == kBuzhash) {
        const BuzFrame f = buz_frame(a.mask);
        a.buz_rot = f.rot;
        a.mask = f.mask;
        a.buz_lim = f.lim;
    }
    a.buz = t.buz;
    a.rk_out = t.rk_out;
    a.rk_mod = t.rk_mod;
    a.rk_shift = static_cast<uint32_t>(tables().rk_shift);
    // largest power of two <= avg / 256, within [256, kLaneMax]: tiles of ~avg/4 (1 MiB and
    // larger averages keep the full 2 KiB lane segments)
    uint64_t cap = algo.kind == kBuzhash ? dev::kBuzLaneMax : dev::kLaneMax;
    while (cap > 256 && cap * dev::kTileDiv > algo.avg) cap >>= 1;
    a.lane_cap = algo.kind == kBuzhash && g_test.lane_cap ? g_test.lane_cap : static_cast<uint32_t>(cap);
    return a;
}
#if KCDC_TRACE || KCDC_DEBUG_CHECKS
char* g_last_ws = nullptr;
#endif
#if KCDC_TRACE
uint64_t* g_trace = nullptr;
uint64_t g_trace_n = 0;
int trace_reserve(uint64_t nstreams) {
    if (g_trace_n >= nstreams) return 0;
    if (g_trace) (void)hipFree(g_trace);
    g_trace = nullptr;
    g_trace_n = 0;
    if (hipMalloc(&g_trace, 3 * 8 * nstreams) != hipSuccess) return -1;
    g_trace_n = nstreams;
    return 0;
}
#endif
}  // namespace

#if KCDC_TRACE || KCDC_DEBUG_CHECKS
// Trace / debug builds only: copy the last launch's queue header.
extern "C" int kcdc_debug_queue_copy(uint32_t* host) {  // the last launch's queue header
    if (!g_last_ws) return -22;
    return hipMemcpy(host, g_last_ws, dev::kQHeaderBytes, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -5;
}
#endif
#if KCDC_TRACE
extern "C" int kcdc_debug_trace_copy(uint64_t* host, uint64_t nstreams) {
    if (!g_trace || nstreams > g_trace_n) return -22;
    return hipMemcpy(host, g_trace, 3 * 8 * nstreams, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -5;
}
#endif

// Experiment switches that make the batch kernels cut WRONG: none are left in the source (round 4
// moved the timing ablations out; kcdc_version, tests/test_lib_host.py).
const char* ablations_kernels() { return ""; }

const DeviceTables* device_tables(int device, int* err) {
    *err = 0;
    if (device < 0 || device >= kMaxDevices) {
        *err = set_error(-22, "device index out of range");
        return nullptr;
    }
    std::lock_guard<std::mutex> lk(g_dev_mu[device]);
    if (g_dev_ready[device]) return &g_dev_tables[device];
    const Tables& T = tables();
    int prev = 0;
    (void)hipGetDevice(&prev);
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) {
        *err = hip_fail(e, "hipSetDevice");
        return nullptr;
    }
    DeviceTables d;
    hipDeviceProp_t prop;
    e = hipGetDeviceProperties(&prop, device);
    if (e == hipSuccess) d.cus = prop.multiProcessorCount;
    if (e == hipSuccess) e = hipMalloc(&d.buz, sizeof(T.buz));
    if (e == hipSuccess) e = hipMalloc(&d.rk_out, sizeof(T.rk_out));
    if (e == hipSuccess) e = hipMalloc(&d.rk_mod, sizeof(T.rk_mod));
    if (e == hipSuccess) e = hipMemcpy(d.buz, T.buz, sizeof(T.buz), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d.rk_out, T.rk_out, sizeof(T.rk_out), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d.rk_mod, T.rk_mod, sizeof(T.rk_mod), hipMemcpyHostToDevice);
    (void)hipSetDevice(prev);
    if (e != hipSuccess) {
        *err = hip_fail(e, "table upload");
        return nullptr;
    }
    g_dev_tables[device] = d;
    g_dev_ready[device] = true;
    return &g_dev_tables[device];
}

int launch_split_batch(const Algo& algo, const SplitArgs& s, int device, void* stream) {
    int err = 0;
    const DeviceTables* t = device_tables(device, &err);
    if (!t) return err;
    if (s.nstreams == 0) return 0;
    dev::BatchArgs a = base_args(algo, *t);
    a.ptrs = s.ptrs;
    a.lens = s.lens;
    a.nstreams = s.nstreams;
    a.cuts = s.cuts;
    a.cuts_cap = s.cuts_cap;
    a.cut_base = s.cut_base;
    a.cut_end = s.cut_end;
    a.starts = s.starts;
    a.resume = s.starts ? s.resume : nullptr;
    a.counts = s.counts;
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (s.starts && algo.kind == kFixed) return set_error(-22, "per-stream starts need the pipelined batch kernels");
    if (algo.kind == kFixed) {
        hipLaunchKernelGGL(dev::split_fixed_kernel, dim3(s.nstreams), dim3(256), 0, st, a);
    } else {
        const unsigned cus = static_cast<unsigned>(t->cus);
        if (algo.kind == kRabinKarp && tables().rk_shift != 45)
            return set_error(-22, "Rabin-Karp kernel: the polynomial must have degree 53");
        const unsigned wg_waves = algo.kind == kRabinKarp ? dev::kRkWaves : dev::kDmaWaves;
        const unsigned need = (s.nstreams + wg_waves - 1) / wg_waves;
        // With helpers the batch kernels take the whole chip even for a few streams: the waves
        // without a stream help scan the owners' regions (help slots).  Help pays when a chunk's
        // test region spans many tiles: averages of 1 MiB and up (12+ buzhash tiles, 6+ Rabin-Karp
        // tiles per region).  Below that, the claims, row waits and helpers' polling cost more than
        // the tail they remove (same-process A/B, 4096 x 4 MiB: 128K-BUZHASH 3.42 vs 3.13 ms with
        // help off, 512K 2.37 vs 2.27; 64 x 64 MiB 128K-BUZHASH 27.5 vs 22.2 ms), except for the
        // Rabin-Karp kernel in launches with fewer streams than waves (64 x 64 MiB 128K-RABINKARP
        // 30.1 vs 38.0 ms); DESIGN.md §2.1d, profiles/r05/help_policy/.
        const bool helpers = g_test.help == 2 ||
                             (g_test.help == 0 &&
                              (algo.avg >= KCDC_HELP_MIN_AVG ||
                               (algo.kind == kRabinKarp && s.nstreams < static_cast<uint64_t>(cus) * wg_waves)));
        unsigned grid = helpers || need >= cus ? cus : need;
        if (grid > dev::kMaxPipeGrid) grid = dev::kMaxPipeGrid;  // one claim flag per workgroup
        // Fewer streams than waves: the waves without a stream of their own live on help tasks
        // (half tiles of the owners' regions), and 4 KiB buzhash lanes (tiles and help tasks twice
        // as long, half the claims, posts and warm-ups per region) win there, while with more
        // streams than waves they lose (the coarser tail).  Same-process A/B,
        // bit-exact, 2 KiB -> 4 KiB (profiles/r06/lane4k/): 4M 2048 x 8 MiB 1.864 -> 1.753 ms,
        // 1024 x 16 MiB 2.855 -> 2.516, 512 x 32 MiB 9.72 -> 7.69; 2M 1024 x 16 MiB 3.09 -> 2.84;
        // 1M loses at 2048 x 8 MiB (2.22 -> 2.29) and gains from 1024 x 16 MiB on (3.67 -> 3.61).
        if (algo.kind == kBuzhash && !g_test.lane_cap && a.lane_cap == dev::kBuzLaneMax && helpers &&
            s.nstreams * (algo.avg >= (2u << 20) ? 1u : 2u) <= static_cast<uint64_t>(grid) * wg_waves)
            a.lane_cap = 2 * dev::kBuzLaneMax;
        // Four or more waves per stream (both batch kernels): helpers outnumber the owners, and regions published
        // four tiles at a time keep them just ahead of the owner instead of on the far end of the
        // region (512 x 32 MiB 4M 7.83 -> 5.89 ms, 1M 8.28 -> 6.93).  With one helper per owner the
        // windows' re-publishing costs more than they save (1024 x 16 MiB 4M 2.49 -> 2.58 at 8
        // tiles, 3.10 at 4), so whole regions stay published there (profiles/r06/help_window/).
        if (g_test.help_window)
            a.help_window = g_test.help_window == 255u ? 0u : g_test.help_window;
        else if (helpers && 4u * s.nstreams <= static_cast<uint64_t>(grid) * wg_waves) {
            // buzhash: wider windows for more helpers per owner (16 waves per stream, 128 x 128 MiB:
            // W = 4 19.9 ms, 6 17.3, 8 18.8; 32 per stream, 64 x 256 MiB: 4 33.4, 6 30.4, 8 27.9)
            const uint64_t wps = static_cast<uint64_t>(grid) * wg_waves / s.nstreams;
            a.help_window = algo.kind == kBuzhash && wps >= 32 ? 8u : algo.kind == kBuzhash && wps >= 16 ? 6u : 4u;
        }
        // Rabin-Karp (a tile is ~2.5x a buzhash tile's time, so re-publishing costs relatively
        // less): windows of 8 tiles pay from one helper per owner on (1024 x 16 MiB 4M 4.52 ->
        // 4.05 ms, 1M 5.56 -> 5.46); with four or more, 4 tiles (512 x 32 MiB 8.17 -> 6.33,
        // 256 x 64 MiB 19.06 -> 11.69; profiles/r06/help_window/rk/)
        else if (algo.kind == kRabinKarp && helpers && 2u * s.nstreams <= static_cast<uint64_t>(grid) * wg_waves)
            a.help_window = 8u;
        uint64_t ring = 1;
        // every push (yields, tombstones) takes a fresh slot; a launch pushes at most
        // a few entries per wave beyond the initial n: size the ring with ample margin
        const uint64_t live = static_cast<uint64_t>(s.nstreams) + 8ull * grid * wg_waves;
        while (ring <= live) ring <<= 1;
        const size_t ring_bytes = static_cast<size_t>(dev::kPEntryStride) * ring;
        const size_t hdr = dev::kQHeaderBytes;
        const uint32_t hwaves = helpers ? grid * wg_waves : 0u;
        const size_t help_bytes = static_cast<size_t>(hwaves) * (128u + 64u + 8u * dev::kHelpTiles) + 4u * ((hwaves + 31u) / 32u);
        const size_t bytes = hdr + ring_bytes + help_bytes;
        char* ws = nullptr;
        // The slot stays locked from its selection to its event record, so a later user of the
        // same slot always waits for this launch.
        std::lock_guard<std::mutex> lk(g_dev_mu[device]);
        unsigned slot = kQueueSlots;
        StreamSlot* aff = nullptr;
        for (StreamSlot& e : g_stream_slot[device]) {
            if (e.valid && e.st == st) aff = &e;
        }
        if (aff && g_qws[device][aff->slot].last == st) slot = aff->slot;
        if (slot == kQueueSlots) {
            slot = g_queue_next[device]++ % kQueueSlots;
            if (!aff) {  // remember this stream in the least recently used entry
                aff = &g_stream_slot[device][0];
                for (StreamSlot& e : g_stream_slot[device])
                    if (!e.valid || e.tick < aff->tick) aff = &e;
                aff->valid = true;
                aff->st = st;
            }
            aff->slot = slot;
        }
        aff->tick = ++g_slot_tick[device];
        QueueWs& q = g_qws[device][slot];
        const bool same_stream = q.used && q.last == st;  // stream order covers the previous launch
        {
            if (q.bytes < bytes) {
                int prev = 0;
                (void)hipGetDevice(&prev);
                (void)hipSetDevice(device);
                char* nb = nullptr;
                size_t nbytes = bytes > 2 * q.bytes ? bytes : 2 * q.bytes;
                // Stream-ordered: a plain hipFree synchronises the whole device, so a launch that
                // grows its slot would wait for every kernel on every stream (tests/test_gpu_queue.py
                // steal test: the batch waited out a 300 ms occupier on another stream).
                hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&nb), nbytes, st);
                if (e == hipSuccess && q.base) {  // the slot's previous launches are the old buffer's only users
                    if (q.done) e = hipStreamWaitEvent(st, q.done, 0);
                    if (e == hipSuccess) e = hipFreeAsync(q.base, st);
                }
                (void)hipSetDevice(prev);
                if (e != hipSuccess) return hip_fail(e, "queue workspace");
                q.base = nb;
                q.bytes = nbytes;
            }
            ws = q.base;
            if (!q.done) {
                int prev = 0;
                (void)hipGetDevice(&prev);
                (void)hipSetDevice(device);
                const hipError_t e = hipEventCreateWithFlags(&q.done, hipEventDisableTiming | hipEventDisableSystemFence);
                (void)hipSetDevice(prev);
                if (e != hipSuccess) return hip_fail(e, "queue workspace event");
            } else if (!same_stream) {
                const hipError_t e = hipStreamWaitEvent(st, q.done, 0);
                if (e != hipSuccess) return hip_fail(e, "queue workspace wait");
            }
            q.last = st;
            q.used = true;
        }
        a.queue = reinterpret_cast<uint32_t*>(ws);
        g_test.last_ws = ws;
        g_test.last_dev = device;
        g_test.last_waves = grid * wg_waves;
#if KCDC_TRACE || KCDC_DEBUG_CHECKS
        g_last_ws = ws;
#endif
        a.ring = reinterpret_cast<uint32_t*>(ws + hdr);
        a.help = helpers ? reinterpret_cast<uint64_t*>(ws + hdr + ring_bytes) : nullptr;
        a.help_waves = hwaves;
        a.ring_mask = static_cast<uint32_t>(ring - 1);

#if KCDC_TRACE
        if (trace_reserve(std::max<uint64_t>(s.nstreams, 3ull * grid * wg_waves)) != 0) return set_error(-12, "trace buffer");
        a.trace = g_trace;
#endif
        // header + ring zeroed per launch (the ring is also left empty by every finished launch)
        {
            const uint32_t slots = static_cast<uint32_t>(ring);
            const uint64_t threads = std::max<uint64_t>(std::max<uint64_t>(8ull * slots, dev::kQHeaderBytes / 4), hwaves);  // >= nstreams
            hipLaunchKernelGGL(dev::init_ring_kernel, dim3(static_cast<unsigned>((threads + 255) / 256)), dim3(256), 0, st, a,
                               slots, grid * wg_waves, g_test.spin_cap ? g_test.spin_cap : dev::kSpinCap,
                               g_test.no_steal ? 0u : dev::kStealSpins);
        }
        // persistent grid: one workgroup per CU, never more workgroups than the streams need
        if (algo.kind == kRabinKarp) {
            hipLaunchKernelGGL(dev::split_batch_rk_kernel, dim3(grid), dim3(dev::kRkWaves * dev::kWave), 0, st, a);
            if (g_test.force_error)
                hipLaunchKernelGGL(dev::poison_counts_kernel, dim3(std::min<unsigned>((s.nstreams + 255) / 256, 256u)),
                                   dim3(256), 0, st, a);
        } else {
            const bool top = buz_frame(static_cast<uint32_t>(algo.mask())).top;
            if (top)
                hipLaunchKernelGGL(dev::split_batch_pipe_kernel<true>, dim3(grid), dim3(dev::kDmaWaves * dev::kWave), 0,
                                   st, a);
            else
                hipLaunchKernelGGL(dev::split_batch_pipe_kernel<false>, dim3(grid), dim3(dev::kDmaWaves * dev::kWave), 0,
                                   st, a);
            if (g_test.force_error)  // test hook: report a failed launch (kcdc_test_set)
                hipLaunchKernelGGL(dev::poison_counts_kernel, dim3(std::min<unsigned>((s.nstreams + 255) / 256, 256u)),
                                   dim3(256), 0, st, a);
        }
        const hipError_t er = hipEventRecord(q.done, st);
        if (er != hipSuccess) return hip_fail(er, "queue workspace record");
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : hip_fail(e, "split kernel launch");
}

int launch_scan_first(const Algo& algo, const uint8_t* d_buf, uint64_t len, int64_t lo, int64_t hi, int64_t* d_out,
                      int device, void* stream, uint8_t* d_scratch) {
    int err = 0;
    const DeviceTables* t = device_tables(device, &err);
    if (!t) return err;
    dev::BatchArgs a = base_args(algo, *t);
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (d_scratch && (algo.kind == kBuzhash || algo.kind == kRabinKarp)) {
        if (algo.kind == kBuzhash)
            hipLaunchKernelGGL(dev::scan_first_cp_kernel<kBuzhash>, dim3(1), dim3(dev::kCpWaves * dev::kWave), 0, st, a,
                               d_buf, static_cast<int64_t>(len), lo, hi, d_out, d_scratch);
        else
            hipLaunchKernelGGL(dev::scan_first_cp_kernel<kRabinKarp>, dim3(1), dim3(dev::kCpWaves * dev::kWave), 0, st,
                               a, d_buf, static_cast<int64_t>(len), lo, hi, d_out, d_scratch);
        const hipError_t e = hipGetLastError();
        return e == hipSuccess ? 0 : hip_fail(e, "scan kernel launch");
    }
    if (algo.kind == kBuzhash)
        hipLaunchKernelGGL(dev::scan_first_kernel<kBuzhash>, dim3(1), dim3(dev::kWave), 0, st, a, d_buf,
                           static_cast<int64_t>(len), lo, hi, d_out);
    else if (algo.kind == kRabinKarp)
        hipLaunchKernelGGL(dev::scan_first_kernel<kRabinKarp>, dim3(1), dim3(dev::kWave), 0, st, a, d_buf,
                           static_cast<int64_t>(len), lo, hi, d_out);
    else
        return set_error(-22, "scan_first: FIXED splitters read no data");
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : hip_fail(e, "scan kernel launch");
}

// ---- resident scan server (host side): one per (device, hash kind)
namespace {
struct ScanServer {
    std::mutex mu;
    bool init = false;
    hipStream_t st = nullptr;
    dev::ServerMbox* h = nullptr;  // fine-grained, mapped
    dev::ServerMbox* d = nullptr;
    uint8_t* scratch = nullptr;
    uint64_t cap = 0;
    uint64_t seq = 0;
    bool launched = false;
    std::chrono::steady_clock::time_point last_answer{};  // the server was alive then
};
ScanServer g_srv[64][2];
bool g_srv_off = false;  // kcdc_test_set(KCDC_TEST_NO_SERVER)
std::atomic<uint64_t> g_srv_served{0};  // requests answered by a server (kcdc_test_server_requests)

int srv_launch(ScanServer& sv, const Algo& algo, const DeviceTables& t) {
    dev::BatchArgs a = base_args(algo, t);
    if (algo.kind == kBuzhash)
        hipLaunchKernelGGL(dev::scan_server_kernel<kBuzhash>, dim3(1), dim3(dev::kSrvWaves * dev::kWave), 0, sv.st, a,
                           sv.d, sv.scratch, sv.seq - 1);
    else
        hipLaunchKernelGGL(dev::scan_server_kernel<kRabinKarp>, dim3(1), dim3(dev::kSrvWaves * dev::kWave), 0, sv.st, a,
                           sv.d, sv.scratch, sv.seq - 1);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "scan server launch");
    sv.launched = true;
    return 0;
}
}  // namespace

void set_scan_server_off(bool off) { g_srv_off = off; }
uint64_t scan_server_requests() { return g_srv_served.load(std::memory_order_relaxed); }

int server_scan_first(const Algo& algo, const uint8_t* d_stage, uint64_t len, int64_t lo, int64_t hi, int device,
                      int64_t* out) {
    if (g_srv_off || device < 0 || device >= 64 || (algo.kind != kBuzhash && algo.kind != kRabinKarp)) return 1;
    ScanServer& sv = g_srv[device][algo.kind == kBuzhash ? 0 : 1];
    std::unique_lock<std::mutex> lk(sv.mu, std::try_to_lock);
    if (!lk.owns_lock()) return 1;  // another handle holds the server: the caller launches its own scan
    int err = 0;
    const DeviceTables* t = device_tables(device, &err);
    if (!t) return err;
    if (!sv.init) {
        if (hipStreamCreateWithFlags(&sv.st, hipStreamNonBlocking) != hipSuccess) return 1;
        void* p = nullptr;
        if (hipHostMalloc(&p, sizeof(dev::ServerMbox), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
            return 1;
        sv.h = static_cast<dev::ServerMbox*>(p);
        std::memset(sv.h, 0, sizeof(dev::ServerMbox));
        void* pd = nullptr;
        if (hipHostGetDevicePointer(&pd, p, 0) != hipSuccess) return 1;
        sv.d = static_cast<dev::ServerMbox*>(pd);
        sv.init = true;
    }
    if (len > sv.cap) {  // grow the scratch: the previous server must be gone first
        if (sv.launched) {
            if (hipStreamSynchronize(sv.st) != hipSuccess) return hip_fail(hipGetLastError(), "scan server sync");
            sv.launched = false;
        }
        if (sv.scratch) (void)hipFree(sv.scratch);
        sv.scratch = nullptr;
        sv.cap = 0;
        const uint64_t cap = std::max<uint64_t>((len + 255) & ~uint64_t(255), 4ull << 20);
        if (hipMalloc(&sv.scratch, cap) != hipSuccess) return 1;
        sv.cap = cap;
    }
    sv.h->src = reinterpret_cast<uint64_t>(d_stage);
    sv.h->len = static_cast<int64_t>(len);
    sv.h->lo = lo;
    sv.h->hi = hi;
    const uint64_t sq = ++sv.seq;
    __atomic_store_n(&sv.h->req_seq, sq, __ATOMIC_RELEASE);
    using clk = std::chrono::steady_clock;
    const auto t_start = clk::now();
    // A server that answered within the last millisecond is still polling (it idles out after
    // 2 ms): skip the runtime query, which costs microseconds.  Otherwise ask the stream.
    if (!sv.launched || (t_start - sv.last_answer > std::chrono::milliseconds(1) && hipStreamQuery(sv.st) == hipSuccess)) {
        const int rc = srv_launch(sv, algo, *t);
        if (rc) return rc;
    }
    // Wait for the answer.  A server that timed out before seeing this request has finished
    // its kernel (hipStreamQuery succeeds) without serving it: launch a new one.
    auto next_check = t_start + std::chrono::microseconds(200);
    uint32_t spins = 0;
    while (__atomic_load_n(&sv.h->done_seq, __ATOMIC_ACQUIRE) != sq) {
        if (++spins % 64 == 0) {
            const auto now = clk::now();
            if (now < next_check) continue;
            next_check = now + std::chrono::microseconds(200);
            if (hipStreamQuery(sv.st) == hipSuccess && __atomic_load_n(&sv.h->done_seq, __ATOMIC_ACQUIRE) != sq) {
                const int rc = srv_launch(sv, algo, *t);
                if (rc) return rc;
            }
            if (now - t_start > std::chrono::seconds(10)) return set_error(-5, "scan server did not answer");
        }
    }
    *out = __atomic_load_n(&sv.h->result, __ATOMIC_ACQUIRE);
    sv.last_answer = clk::now();
    g_srv_served.fetch_add(1, std::memory_order_relaxed);
    return 0;
}

int launch_scan_first_batch(const Algo& algo, const uint8_t* d_base, const ScanReq* d_reqs, uint32_t n, int64_t* d_out,
                            int device, void* stream, uint8_t* d_scratch) {
    int err = 0;
    const DeviceTables* t = device_tables(device, &err);
    if (!t) return err;
    if (n == 0) return 0;
    dev::BatchArgs a = base_args(algo, *t);
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (d_scratch && (algo.kind == kBuzhash || algo.kind == kRabinKarp)) {
        if (algo.kind == kBuzhash)
            hipLaunchKernelGGL(dev::scan_first_batch_cp_kernel<kBuzhash>, dim3(n), dim3(dev::kCpWaves * dev::kWave), 0,
                               st, a, d_base, d_reqs, d_out, d_scratch);
        else
            hipLaunchKernelGGL(dev::scan_first_batch_cp_kernel<kRabinKarp>, dim3(n), dim3(dev::kCpWaves * dev::kWave), 0,
                               st, a, d_base, d_reqs, d_out, d_scratch);
        const hipError_t e = hipGetLastError();
        return e == hipSuccess ? 0 : hip_fail(e, "scan kernel launch");
    }
    if (algo.kind == kBuzhash)
        hipLaunchKernelGGL(dev::scan_first_batch_kernel<kBuzhash>, dim3(n), dim3(dev::kWave), 0, st, a, d_base, d_reqs,
                           d_out);
    else if (algo.kind == kRabinKarp)
        hipLaunchKernelGGL(dev::scan_first_batch_kernel<kRabinKarp>, dim3(n), dim3(dev::kWave), 0, st, a, d_base,
                           d_reqs, d_out);
    else
        return set_error(-22, "scan_first: FIXED splitters read no data");
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : hip_fail(e, "scan kernel launch");
}

int launch_fill_prng(uint8_t* d_data, uint64_t stride, uint64_t stream_len, uint32_t nstreams, uint64_t seed,
                     uint64_t first_sid, void* stream) {
    if (stride % 8 != 0 || (nstreams > 1 && stride < stream_len))
        return set_error(-22, "fill_prng: stride must be a multiple of 8 and >= stream_len");
    if (nstreams == 0 || stream_len == 0) return 0;
    hipLaunchKernelGGL(dev::fill_prng_kernel, dim3(4096), dim3(256), 0, static_cast<hipStream_t>(stream), d_data,
                       stride, stream_len, nstreams, seed, first_sid);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : hip_fail(e, "fill kernel launch");
}

namespace {
constexpr uint64_t kParNodeCap = uint64_t(1) << 20;  // parallel-resolver nodes per launch (<= 88 MB of tables)
struct LongLayout {
    int64_t nseg;
    uint64_t node_cap;
    uint32_t levels;
    size_t off_streams, off_cnt, off_cand, off_off, off_list, off_total, off_bsum, off_serial, off_forced, off_jump, bytes;
};
int64_t long_nseg(uint64_t len, uint64_t off0) {  // segments tile coordinates (position + off0)
    return len ? static_cast<int64_t>((len + off0 + dev::kSegBytes - 1) / dev::kSegBytes) : 0;
}
LongLayout long_layout(int64_t nseg, uint32_t nstreams) {
    auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
    LongLayout L{};
    L.nseg = nseg;
    const size_t ns = static_cast<size_t>(nseg);
    size_t o = 0;
    L.off_streams = o;
    o += al(nstreams * sizeof(dev::LongStream));
    L.off_cnt = o;
    o += al(ns * 4);
    L.off_cand = o;
    o += al(ns * dev::kSegK * 8);
    L.off_off = o;
    o += al(ns * 8);
    L.off_list = o;
    o += al(ns * dev::kSegK * 8);
    L.off_total = o;
    o += 256;
    L.off_bsum = o;
    o += al((static_cast<size_t>(nseg) + dev::kPrefixItems - 1) / dev::kPrefixItems * 8 + 8);
    L.node_cap = 0;
    L.levels = 0;
    L.off_serial = L.off_forced = L.off_jump = o;
    {  // resolve_par_kernel for streams with complete candidate lists
        L.node_cap = std::min<uint64_t>(static_cast<uint64_t>(ns) * dev::kSegK + 2ull * nstreams, kParNodeCap);
        L.levels = 1;
        while ((uint64_t(1) << L.levels) <= L.node_cap) L.levels++;
        L.off_serial = o;
        o += al(nstreams * 4);
        L.off_forced = o;
        o += al(L.node_cap * 4);
        L.off_jump = o;
        o += al(static_cast<size_t>(L.levels) * L.node_cap * 4);
    }
    L.bytes = o;
    return L;
}
}  // namespace

size_t long_workspace_bytes(const Algo& algo, uint64_t len) {
    if (algo.kind == kFixed) return 0;
    return long_layout(long_nseg(len, 15), 1).bytes;  // any alignment: off0 < 16
}

size_t long_workspace_bytes_multi(const Algo& algo, const uint64_t* lens, uint32_t m) {
    if (algo.kind == kFixed) return 0;
    int64_t nseg = 0;
    for (uint32_t j = 0; j < m; j++) nseg += long_nseg(lens[j], 15);
    return long_layout(nseg, m).bytes;
}

int launch_split_long_multi(const Algo& algo, uint32_t m, const uint8_t* const* d_data, const uint64_t* lens,
                            uint64_t* const* d_cuts, const uint64_t* caps, uint64_t* const* d_counts, void* ws,
                            size_t ws_bytes, int device, void* stream) {
    int err = 0;
    const DeviceTables* t = device_tables(device, &err);
    if (!t) return err;
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (algo.kind == kFixed)  // reads no data; the batch entry point covers it
        return set_error(-22, "long-stream path: use kcdc_split_batch_device for FIXED splitters");
    if (m == 0) return 0;
    std::vector<dev::LongStream> hs(m);
    int64_t nseg = 0;
    for (uint32_t j = 0; j < m; j++) {
        const uint64_t p = reinterpret_cast<uint64_t>(d_data[j]);
        dev::LongStream& S = hs[j];
        S.off0 = static_cast<int64_t>(p & 15u);
        S.abase = reinterpret_cast<const uint8_t*>(p - static_cast<uint64_t>(S.off0));
        S.n = static_cast<int64_t>(lens[j]);
        S.seg0 = nseg;
        S.cuts = d_cuts[j];
        S.cuts_cap = caps[j];
        S.count = d_counts[j];
        nseg += long_nseg(lens[j], static_cast<uint64_t>(S.off0));
    }
    const LongLayout L = long_layout(nseg, m);
    if (!ws || ws_bytes < L.bytes) return set_error(-22, "long-stream path: workspace too small");
    char* w = static_cast<char*>(ws);
    dev::LongArgs g{};
    g.streams = reinterpret_cast<const dev::LongStream*>(w + L.off_streams);
    g.nstreams = m;
    g.nseg = nseg;
    g.seg_cnt = reinterpret_cast<uint32_t*>(w + L.off_cnt);
    g.seg_cand = reinterpret_cast<uint64_t*>(w + L.off_cand);
    g.seg_off = reinterpret_cast<uint64_t*>(w + L.off_off);
    g.list = reinterpret_cast<uint64_t*>(w + L.off_list);
    g.total = reinterpret_cast<uint64_t*>(w + L.off_total);
    {
        g.serial = reinterpret_cast<uint32_t*>(w + L.off_serial);
        g.forced = reinterpret_cast<uint32_t*>(w + L.off_forced);
        g.jump = reinterpret_cast<uint32_t*>(w + L.off_jump);
        g.node_cap = L.node_cap;
        g.levels = L.levels;
    }
    hipError_t e = hipMemcpyAsync(w + L.off_streams, hs.data(), m * sizeof(dev::LongStream), hipMemcpyHostToDevice, st);
    if (e != hipSuccess) return hip_fail(e, "long-stream descriptors");
    dev::BatchArgs a = base_args(algo, *t);
    const int64_t mn = static_cast<int64_t>(algo.min_size()), mx = static_cast<int64_t>(algo.max_size());
    if (nseg > 0) {
        if (algo.kind == kBuzhash) {  // LDS-DMA fed, persistent: one workgroup per CU
            const dim3 pgrid(static_cast<unsigned>(
                std::min<int64_t>(t->cus, (nseg + dev::kDmaWaves - 1) / dev::kDmaWaves)));
            if (buz_frame(static_cast<uint32_t>(algo.mask())).top)
                hipLaunchKernelGGL(dev::cand_scan_dma_kernel<true>, pgrid, dim3(dev::kDmaWaves * dev::kWave), 0, st, a, g);
            else
                hipLaunchKernelGGL(dev::cand_scan_dma_kernel<false>, pgrid, dim3(dev::kDmaWaves * dev::kWave), 0, st, a, g);
        } else {  // Rabin-Karp: two-chain LDS-DMA tiles, persistent
            const dim3 pgrid(static_cast<unsigned>(
                std::min<int64_t>(t->cus, (nseg + dev::kRkWaves - 1) / dev::kRkWaves)));
            hipLaunchKernelGGL(dev::cand_scan_rk_kernel, pgrid, dim3(dev::kRkWaves * dev::kWave), 0, st, a, g);
        }
        const unsigned nblk = static_cast<unsigned>((nseg + dev::kPrefixItems - 1) / dev::kPrefixItems);
        uint64_t* bsum = reinterpret_cast<uint64_t*>(w + L.off_bsum);
        hipLaunchKernelGGL(dev::seg_blocksum_kernel, dim3(nblk), dim3(1024), 0, st, g, bsum);
        hipLaunchKernelGGL(dev::block_offsets_kernel, dim3(1), dim3(64), 0, st, g, bsum, nblk);
        hipLaunchKernelGGL(dev::seg_prefix_kernel, dim3(nblk), dim3(1024), 0, st, g, bsum);
        hipLaunchKernelGGL(dev::compact_kernel, dim3(static_cast<unsigned>((nseg + 255) / 256)), dim3(256), 0, st, g);
    }
    if (g.serial) {  // streams it cannot take (truncated segments) stay flagged for resolve_kernel
        if (nseg == 0) {
            e = hipMemsetAsync(w + L.off_total, 0, sizeof(uint64_t), st);
            if (e != hipSuccess) return hip_fail(e, "long-stream total");
        }
        hipLaunchKernelGGL(dev::resolve_par_kernel, dim3(m), dim3(1024), 0, st, g, mn, mx);
    }
    if (algo.kind == kBuzhash)
        hipLaunchKernelGGL(dev::resolve_kernel<kBuzhash>, dim3(m), dim3(dev::kWave), 0, st, a, g, mn, mx);
    else
        hipLaunchKernelGGL(dev::resolve_kernel<kRabinKarp>, dim3(m), dim3(dev::kWave), 0, st, a, g, mn, mx);
    e = hipGetLastError();
    return e == hipSuccess ? 0 : hip_fail(e, "long-stream kernel launch");
}

int launch_split_long(const Algo& algo, const uint8_t* d_data, uint64_t len, uint64_t* d_cuts, uint64_t cuts_cap,
                      uint64_t* d_count, void* ws, size_t ws_bytes, int device, void* stream) {
    return launch_split_long_multi(algo, 1, &d_data, &len, &d_cuts, &cuts_cap, &d_count, ws, ws_bytes, device,
                                   stream);
}

// ------------------------------------------------------------------ testing
extern "C" int64_t kcdc_test_server_requests(void) { return static_cast<int64_t>(scan_server_requests()); }

extern "C" int kcdc_test_set(int32_t key, int64_t value) {
    switch (key) {
        case 1: g_test.spin_cap = static_cast<uint32_t>(value); return 0;   // KCDC_TEST_SPIN_CAP
        case 2: g_test.no_steal = value != 0; return 0;                     // KCDC_TEST_NO_STEAL
        case 3: g_test.force_error = value != 0; return 0;                  // KCDC_TEST_FORCE_ERROR
        case 4: test_hash_lanes() = static_cast<int>(value); return 0;     // KCDC_TEST_HASH_LANES
        case 5: set_scan_server_off(value != 0); return 0;                 // KCDC_TEST_NO_SERVER
        case 6: g_test.help = value == 2 ? 2 : value != 0; return 0;       // KCDC_TEST_NO_HELP (2: force help on)
        case 7: test_id_ring_bytes() = static_cast<uint64_t>(value); return 0;  // KCDC_TEST_ID_RING
        case 8:                                                            // KCDC_TEST_LANE_CAP
            if (value != 0 && (value < 256 || value > 4096 || (value & (value - 1)) != 0))
                return set_error(-22, "lane cap: 0, or a power of two in [256, 4096]");
            g_test.lane_cap = static_cast<uint32_t>(value);
            return 0;
        case 9:                                                            // KCDC_TEST_HELP_WINDOW
            if (value < 0 || (value != 0 && (value < static_cast<int64_t>(dev::kHelpMinTiles) || value > 255)))
                return set_error(-22, "help window: 0 (policy), 255 (whole regions), or tiles in [3, 254]");
            g_test.help_window = static_cast<uint32_t>(value);
            return 0;
        default: return set_error(-22, "unknown test knob");
    }
}

extern "C" int64_t kcdc_test_queue_stat(int32_t key) {
    if (key == 12) return g_test.last_ws ? static_cast<int64_t>(g_test.last_waves) : set_error(-22, "no pipelined batch launch yet");
    const int word = key == 1 ? dev::kQErr : key == 2 ? dev::kQDone : key == 3 ? dev::kQSteal : key == 4 ? dev::kQHelp
                   : key >= 5 && key <= 9 ? dev::kQDiag + (key - 5)
                   : key == 10 ? dev::kQHT : key == 11 ? dev::kQHT + 1 : -1;
    if (word < 0) return set_error(-22, "unknown queue statistic");
    if (!g_test.last_ws) return set_error(-22, "no pipelined batch launch yet");
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(g_test.last_dev);
    uint32_t v = 0;
    const hipError_t e = hipMemcpy(&v, g_test.last_ws + 4 * word, 4, hipMemcpyDeviceToHost);
    (void)hipSetDevice(prev);
    return e == hipSuccess ? static_cast<int64_t>(v) : hip_fail(e, "queue statistic");
}

// Test hook: bytes [off, off + n) of the last pipelined launch's queue workspace (header, ring,
// help slots) to host memory, for post-mortems of a launch (tools/batch_probe.py).
extern "C" int kcdc_test_ws_copy(void* dst, uint64_t off, uint64_t n) {
    if (!g_test.last_ws) return set_error(-22, "no pipelined batch launch yet");
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(g_test.last_dev);
    const hipError_t e = hipMemcpy(dst, g_test.last_ws + off, n, hipMemcpyDeviceToHost);
    (void)hipSetDevice(prev);
    return e == hipSuccess ? 0 : hip_fail(e, "workspace copy");
}

extern "C" int kcdc_test_occupy(uint32_t nwg, uint32_t usec, void* stream) {
    if (nwg == 0) return 0;
    if (usec > 10u * 1000u * 1000u) return set_error(-22, "occupy: at most 10 s");
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(dev::occupy_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return hip_fail(e, "occupy attribute");
    uint32_t* sink = nullptr;
    e = hipMallocAsync(reinterpret_cast<void**>(&sink), 4, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return hip_fail(e, "occupy sink");
    hipLaunchKernelGGL(dev::occupy_kernel, dim3(nwg), dim3(64), 160 * 1024, static_cast<hipStream_t>(stream),
                       static_cast<uint64_t>(usec) * 100u, sink);
    e = hipGetLastError();
    (void)hipFreeAsync(sink, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? 0 : hip_fail(e, "occupy launch");
}

}  // namespace kcdc
