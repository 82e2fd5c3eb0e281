// Batching object writers (the writer-level remainder): many concurrent
// objectWriter.Write streams (repo/object/object_writer.go:113-139) fed in 64 KiB slices
// (snapshot/upload/upload.go:394-407) are staged per writer in pinned host blocks and split
// together: one round = one gather launch that pulls every writer's new bytes over PCIe into its
// device arena, one batch-splitter launch over all writers' unresolved regions, their cut lists
// back.  Each byte crosses PCIe once.
//
// Device layout: every writer owns an arena in HBM holding its stream contiguously from the
// window before its last final cut (the chunk in progress) up to the bytes shipped so far; arena
// offset = stream position - origin, origin a multiple of 16.  Host blocks place each byte at a
// block offset congruent to its stream position mod 16, so the gather copies 16-byte vectors.
// Rounds are pipelined: round k+1's gather (new bytes, past round k's regions) runs while round
// k splits; round k+1's launch waits for round k's cuts (its chunk starts).
//
// Exactness: the rolling hash at position p is a function of the 64 bytes ending at p
// (SURVEY.md §0.4), and a chunk's cut is the first candidate in [s+min-1, s+max-1] (or the
// forced cut).  A round splits region [tail_pos, shipped) starting its first chunk at the
// writer's last final cut (kernel `starts`: the bytes before it are window history only), and
// skips the positions the previous round already tested for that chunk (kernel `resume`).
// Every cut it reports is final except the last one, which is the region end (the chunk still
// growing), unless the writer is finishing.  So the cuts equal one NextSplitPoint pass over the
// whole object, however the bytes were sliced (tests/test_gpu_writer.py).
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/kcdc.h"
#include "kcdc_internal.h"

using namespace kcdc;

namespace {

constexpr size_t kBlock = 4u << 20;    // pinned staging block
constexpr size_t kSlabBlocks = 8;      // blocks per pinned allocation
constexpr uint64_t kHist = 64;         // window history kept before a writer's last final cut
constexpr uint32_t kTask = 64u << 10;  // gather: bytes per workgroup

int hip_err(hipError_t e, const char* what) { return set_error(KCDC_EIO, std::string(what) + ": " + hipGetErrorString(e)); }

struct Guard {
    int prev = -1;
    explicit Guard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~Guard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// One gather piece: len bytes from pinned host memory (device-visible) to a writer's arena;
// src and dst are congruent mod 16.
struct Piece {
    const uint8_t* src;
    uint8_t* dst;
    uint64_t len;
    uint64_t task0;  // first 64 KiB task of this piece (exclusive prefix over pieces)
};

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) v4u gv4u;
typedef __attribute__((address_space(1))) uint8_t gu8;

// A bounded grid (kGatherWGs workgroups, grid-stride over 64 KiB tasks): the gather needs few
// CUs to saturate PCIe, and a grid of one workgroup per task filled the machine, so the split
// launch queued behind it and the two never overlapped.  Per task: the bytes before the first
// 16-byte boundary and after the last one singly, the rest as 16-byte vectors, four in flight
// per thread (the reads cross PCIe: latency, not bandwidth, limits one workgroup).
constexpr unsigned kGatherWGs = 96;
__global__ __launch_bounds__(256) void bw_gather_kernel(const Piece* pieces, uint32_t npieces, uint64_t ntasks) {
    for (uint64_t task = blockIdx.x; task < ntasks; task += gridDim.x) {
        uint32_t lo = 0, hi = npieces;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (pieces[mid].task0 <= task) lo = mid;
            else hi = mid;
        }
        const Piece pc = pieces[lo];
        const uint64_t off = (task - pc.task0) * kTask;
        if (off >= pc.len) continue;
        const uint64_t len = pc.len - off < kTask ? pc.len - off : kTask;
        // global, not flat, accesses (the pinned host blocks are mapped into the device's address space)
        const gu8* s = reinterpret_cast<const gu8*>(reinterpret_cast<uintptr_t>(pc.src) + off);
        gu8* d = reinterpret_cast<gu8*>(reinterpret_cast<uintptr_t>(pc.dst) + off);
        const uint32_t head = static_cast<uint32_t>((16u - ((reinterpret_cast<uintptr_t>(pc.dst) + off) & 15u)) & 15u);
        const uint32_t h = head < len ? head : static_cast<uint32_t>(len);
        const uint32_t t = threadIdx.x;
        if (t < h) d[t] = s[t];
        const uint64_t nv = (len - h) / 16;
        const gv4u* sv = reinterpret_cast<const gv4u*>(s + h);
        gv4u* dv = reinterpret_cast<gv4u*>(d + h);
        for (uint64_t i = t; i < nv; i += 4 * 256) {
            v4u v[4];
#pragma unroll
            for (int k = 0; k < 4; k++)
                if (i + 256 * k < nv) v[k] = __builtin_nontemporal_load(sv + i + 256 * k);
#pragma unroll
            for (int k = 0; k < 4; k++)
                if (i + 256 * k < nv) dv[i + 256 * k] = v[k];
        }
        const uint64_t done = h + 16 * nv;
        if (t < len - done) d[done + t] = s[done + t];
    }
}

// The content IDs' ring copies: chunk bytes from any source address to a 16-byte aligned ring
// slot (the chain kernel loads whole aligned vectors).  Per thread 16 destination bytes from five
// aligned source words (never past the source's last word: the next word may not be mapped);
// the last vector of a chunk may write up to 15 bytes past its end, inside the slot (the ring
// reserves each chunk's length rounded up to 16).
__global__ __launch_bounds__(256) void bw_realign_kernel(const Piece* pieces, uint32_t npieces, uint64_t ntasks) {
    for (uint64_t task = blockIdx.x; task < ntasks; task += gridDim.x) {
        uint32_t lo = 0, hi = npieces;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (pieces[mid].task0 <= task) lo = mid;
            else hi = mid;
        }
        const Piece pc = pieces[lo];
        const uint64_t off = (task - pc.task0) * kTask;
        if (off >= pc.len) continue;
        const uint64_t len = pc.len - off < kTask ? pc.len - off : kTask;
        const uintptr_t sa = reinterpret_cast<uintptr_t>(pc.src) + off;
        const uint32_t mis = static_cast<uint32_t>(sa & 3u);
        const __attribute__((address_space(1))) uint32_t* sw =
            reinterpret_cast<const __attribute__((address_space(1))) uint32_t*>(sa - mis);
        gv4u* dv = reinterpret_cast<gv4u*>(reinterpret_cast<uintptr_t>(pc.dst) + off);
        const uint64_t lw = (len + mis - 1) >> 2;  // the last source word holding a chunk byte
        const uint64_t nv = (len + 15) >> 4;
        for (uint64_t i = threadIdx.x; i < nv; i += 256) {
            uint32_t x[5];
#pragma unroll
            for (int k = 0; k < 5; k++) x[k] = sw[4 * i + k < lw ? 4 * i + k : lw];
            v4u o;
            o.x = mis ? __builtin_amdgcn_alignbit(x[1], x[0], 8 * mis) : x[0];
            o.y = mis ? __builtin_amdgcn_alignbit(x[2], x[1], 8 * mis) : x[1];
            o.z = mis ? __builtin_amdgcn_alignbit(x[3], x[2], 8 * mis) : x[2];
            o.w = mis ? __builtin_amdgcn_alignbit(x[4], x[3], 8 * mis) : x[3];
            dv[i] = o;
        }
    }
}

struct Blk {  // a pinned block: bytes [start, end) are stream bytes [pos, pos + end - start)
    uint8_t* p = nullptr;
    uint32_t start = 0, end = 0;
    uint64_t pos = 0;
};

// Staging copy of a writer's slice into its pinned block.  Non-temporal stores write the block
// without first reading its lines (a plain memcpy's stores read each destination line for
// ownership: three memory passes instead of two), and the block is read next by the GPU, not the
// CPU.  With more writer threads than cores the copies are what the host's memory bandwidth goes
// to.  The stores are weakly ordered: the sfence makes them visible before the writer publishes
// the bytes (under its mutex) to the round thread, whose gather reads them over PCIe.
__attribute__((target("avx2"))) void copy_nt_avx2(uint8_t* d, const uint8_t* s, size_t n) {
    const size_t h = std::min<size_t>(n, (32 - (reinterpret_cast<uintptr_t>(d) & 31)) & 31);
    std::memcpy(d, s, h);
    d += h;
    s += h;
    n -= h;
    for (; n >= 128; n -= 128, d += 128, s += 128) {
        const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s));
        const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + 32));
        const __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + 64));
        const __m256i e = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + 96));
        _mm256_stream_si256(reinterpret_cast<__m256i*>(d), a);
        _mm256_stream_si256(reinterpret_cast<__m256i*>(d + 32), b);
        _mm256_stream_si256(reinterpret_cast<__m256i*>(d + 64), c);
        _mm256_stream_si256(reinterpret_cast<__m256i*>(d + 96), e);
    }
    std::memcpy(d, s, n);
    _mm_sfence();
}
const bool g_have_avx2 = __builtin_cpu_supports("avx2");
void stage_copy(uint8_t* d, const uint8_t* s, size_t n) {
    if (g_have_avx2 && n >= 4096) copy_nt_avx2(d, s, n);
    else std::memcpy(d, s, n);
}

int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

}  // namespace

struct kcdc_bw;

// One device's batcher: its round thread, streams, pinned blocks and round metadata.  A
// kcdc_bw_batcher holds one per device of its device set and assigns each writer to one.
struct BwDev {
    const Algo* algo = nullptr;
    int device = 0;
    int index = 0;                     // position in the batcher's device list
    std::atomic<uint64_t> load{0};     // assignment load: max(size hint, bytes written) over open writers
    uint64_t round_bytes = 0;  // ship once this many new bytes are staged across writers
    uint64_t writer_cap = 0;   // a writer blocks in write() while this many of its bytes are unshipped
    uint64_t arena_cap = 0;    // device bytes per writer
    std::chrono::microseconds wait{0};
    hipStream_t stream = nullptr, copy = nullptr;

    std::mutex mu;                     // open list, writer cut state (lock order: mu, then a writer's mu, then pool_mu)
    std::mutex pool_mu;                // the pinned block pool (writers take blocks without the round thread's mutex)
    std::condition_variable cv_round;  // round thread: work arrived
    std::condition_variable cv_done;   // finishing writers: a round completed
    std::vector<kcdc_bw*> open;        // writers not yet freed
    std::vector<uint8_t*> pool;        // free pinned blocks (carved from slabs)
    std::vector<uint8_t*> slabs;       // pinned allocations of kSlabBlocks blocks each
    // arenas of freed writers (arena, spare), reused by the next kcdc_bw_open: an uploader opens a
    // writer per object, and hipMalloc/hipFree of two arenas per object would serialise on the device.
    // The cache holds at most as many pairs as writers were open at once since it was last trimmed
    // (a freed writer's pair waits for the next open; the device never holds more arena memory than
    // that peak needed), and kcdc_bw_open frees it before it reports KCDC_ENOMEM.
    std::vector<std::pair<uint8_t*, uint8_t*>> arenas;
    size_t peak_open = 0;  // (mu) most writers open at once since the cache was last trimmed
    size_t keep_arenas() const { return peak_open; }
    void trim_arenas() {  // mu held; the cached pairs are idle (their writers' rounds completed)
        Guard g(device);
        for (auto& ar : arenas) {
            (void)hipFree(ar.first);
            (void)hipFree(ar.second);
        }
        arenas.clear();
        peak_open = open.size();
    }
    std::atomic<uint64_t> staged{0};   // unshipped bytes over all writers
    std::atomic<int64_t> since{0};     // when `staged` last became nonzero (steady ns)
    std::atomic<uint32_t> capped{0};   // writers blocked on their staging cap (a round is due)
    std::atomic<uint32_t> finish_pending{0};  // finishing writers whose last region is not issued
    uint64_t rounds = 0;
    // (mu) the round thread holds writer pointers outside mu: a round being collected and issued,
    // or id_create reading arenas.  kcdc_bw_free of a writer that may still be in such a round (its
    // last round did not complete: an error) waits until this is 0 before it frees the writer.
    int writer_refs = 0;
    void unref_writers() {  // mu held
        writer_refs--;
        cv_done.notify_all();
    }
    bool stop = false;
    std::atomic<int> error{0};
    std::string errmsg;
    std::thread th;

    // per-round device/pinned metadata, two sets (round k+1 is built while round k is in flight)
    struct Meta {
        uint64_t* d = nullptr;  // ptrs | lens | starts | cut_base | resume | counts | cuts
        uint64_t* h = nullptr;  // pinned mirror
        size_t cap = 0;         // words
        Piece* dp = nullptr;    // gather pieces
        Piece* hp = nullptr;
        size_t pcap = 0;
        hipEvent_t gathered = nullptr, g0 = nullptr, k0 = nullptr, done = nullptr;
    } meta[2];

    // observability (kcdc_bw_stats)
    uint64_t shipped_bytes = 0;
    double t_submit = 0, t_wait = 0, t_gather = 0, t_kernel = 0;
    double t_seg[5] = {0, 0, 0, 0, 0};  // host seconds per round phase: collect, place, gather issue, wait, launch
    hipEvent_t ev_ref = nullptr;                   // recorded once: the origin of the intervals below
    std::vector<std::pair<float, float>> busy;     // device intervals (ms after ev_ref) of gathers and splits
    double t_idle = 0;                             // round thread: waiting for a round's worth of bytes
    std::atomic<int64_t> w_capped_ns{0};           // writers: blocked on their staging cap (summed)
    std::atomic<int64_t> w_block_ns{0};            // writers: getting a pinned block (summed)
    std::atomic<uint64_t> pool_misses{0};          // pinned slabs allocated (the pool was empty)
    double t_lock = 0;                             // round thread: acquiring mu to apply a round

    // ---- content IDs (kcdc_bw_batcher_hash): every final chunk's keyed hash, computed on the
    // device from the bytes the round already holds (content_manager.go:812 hashes each chunk the
    // object writer flushes).  At a round's completion the round thread copies each new final chunk
    // from the writer's arena into the ID ring (copy stream, ordered after that round's compactions)
    // and publishes a chain for it.  A hash thread of its own advances the chains in slices on the
    // hash stream, two steps in flight so the stream never idles between them (a BLAKE2 chunk is one
    // long dependent chain: throughput = chains in flight x one chain's rate, so the ring must stay
    // full and the steps back to back).  Ring bytes and chain slots are reused first in, first out.
    struct IdCfg {
        bool on = false;
        std::string name;
        std::vector<uint8_t> key;
        uint32_t out = 0;  // digest bytes
        int kind = 0;      // 1 BLAKE2b, 2 BLAKE2s (sliced chains), 3 other names (whole chunks per step)
    } ids;
    struct Chain {
        kcdc_bw* w;            // null once its writer was freed
        uint64_t wseq;         // the writer's ID entry
        uint64_t ring_at;      // bytes in the ring (monotonic offset; position = ring_at % ring_cap)
        uint64_t ring_end;     // the ring's monotonic offset after this chain (its bytes and any wrap skip)
        uint64_t len, nblk, done;  // chunk bytes; message blocks; blocks done after the steps issued
        bool fin = false;      // its digest has been delivered
        uint64_t pub = 0;      // its publish (a step takes it once that publish's ring copies are done)
    };
    struct NewChunk {
        kcdc_bw* w;
        uint64_t wseq, pos, len;
    };
    struct Step {  // one hash step's host-side buffers (two steps may be in flight)
        hipEvent_t t0 = nullptr, ev = nullptr;
        uint8_t* h_dig = nullptr;  // digests: by slot (kinds 1, 2) or by position in the step (kind 3)
        uint32_t* h_act = nullptr; // active chain slots
        uint64_t* h_ol = nullptr;  // kind 3: ring offsets, then lengths
        std::vector<std::pair<uint64_t, uint32_t>> done;  // (chain number, digest row) ending in this step
    } steps[2];
    std::vector<NewChunk> newc;        // final chunks of the last completed round (round thread)
    hipStream_t hstream = nullptr;
    uint8_t* ring = nullptr;
    // monotonic byte offsets; ring_head: round thread (reservations), ring_tail: hash thread (mu)
    uint64_t ring_cap = 0, ring_head = 0, ring_tail = 0;
    HashChain* d_chains = nullptr;
    HashChain* h_chains = nullptr;     // pinned: new chains' records, by slot (round thread writes, hash thread uploads)
    uint32_t chain_cap = 0;
    // monotonic chain numbers (mu): [chain_tail, chain_head) published
    uint64_t chain_head = 0, chain_tail = 0;
    uint64_t undone = 0;               // (mu) published chains with blocks not yet issued
    std::deque<Chain> chains;          // chains [chain_tail, chain_head)
    uint8_t* d_dig = nullptr;
    uint32_t* d_act = nullptr;
    uint64_t* d_ol = nullptr;
    // Ring copies run on their own stream (idcopy): behind the compactions of the last collected
    // round (compacted_ev, recorded on the copy stream before that round's gather), not behind the
    // gather itself, so hash steps never wait for PCIe.  Compactions in turn wait for the ring
    // copies issued so far (copy_ev): a compaction may overwrite an arena the copies read.
    hipStream_t idcopy = nullptr;
    hipEvent_t copy_ev = nullptr;      // the ring copies of the chains published so far (idcopy)
    hipEvent_t compacted_ev = nullptr; // the compactions of the last collected round (copy stream)
    // One event per publish (a ring of kPubEv): a step takes only chains whose copies are known
    // done, so the hash stream never waits on the copies (they wait on compactions, which sit
    // behind a gather on the copy stream).
    static constexpr uint64_t kPubEv = 64;
    static constexpr uint64_t kPubPieces = 1024;  // chunks per publish (one copy launch each)
    hipEvent_t pub_ev[kPubEv] = {};
    Piece* h_rp = nullptr;             // pinned: publish seq's copy pieces at slot seq % kPubEv
    Piece* d_rp = nullptr;
    uint64_t pub_seq = 0, pub_done = 0;  // (mu) publishes issued; [0, pub_done) known complete
    uint64_t step_blocks = 0;
    uint64_t id_chains = 0, id_steps = 0;
    double t_hash = 0;                 // device seconds of the hash steps
    double t_space = 0;                // round thread: seconds waiting for ring space / chain slots
    double t_hidle = 0;                // hash thread: seconds with no step in flight
    uint64_t chain_steps = 0;          // chains advanced, summed over steps (/ id_steps: chains per step)
    std::condition_variable cv_hash;   // hash thread: chains published, or stop
    std::condition_variable cv_space;  // round thread: ring space or chain slots freed
    bool hstop = false;                // (mu) the round thread has published its last chains
    std::thread hth;
    int ids_enable(const char* name, const uint8_t* key, uint32_t key_len);
    void ids_disable();                // undo ids_enable (no writer has opened yet)
    int id_create();                   // round thread, mu not held: newc -> chains (ring copies)
    int id_issue(Step& st, bool& issued);  // hash thread, mu not held
    int id_deliver(Step& st);          // hash thread, mu not held
    void hash_loop();
    void fail(int rc);                 // mu not held: record the first error, wake everyone

    ~BwDev() {
        if (hth.joinable()) {  // (a batcher whose round thread never started it cleanly)
            {
                std::lock_guard<std::mutex> lk(mu);
                hstop = true;
            }
            cv_hash.notify_all();
            hth.join();
        }
        if (algo->kind == kFixed) return;
        Guard g(device);
        for (uint8_t* s : slabs) (void)hipHostFree(s);
        for (auto& a : arenas) {
            (void)hipFree(a.first);
            (void)hipFree(a.second);
        }
        for (Meta& m : meta) {
            if (m.d) (void)hipFree(m.d);
            if (m.h) (void)hipHostFree(m.h);
            if (m.dp) (void)hipFree(m.dp);
            if (m.hp) (void)hipHostFree(m.hp);
            for (hipEvent_t e : {m.gathered, m.g0, m.k0, m.done})
                if (e) (void)hipEventDestroy(e);
        }
        if (ev_ref) (void)hipEventDestroy(ev_ref);
        if (copy_ev) (void)hipEventDestroy(copy_ev);
        if (h_rp) (void)hipHostFree(h_rp);
        if (d_rp) (void)hipFree(d_rp);
        for (hipEvent_t ev : pub_ev)
            if (ev) (void)hipEventDestroy(ev);
        if (compacted_ev) (void)hipEventDestroy(compacted_ev);
        if (idcopy) (void)hipStreamDestroy(idcopy);
        for (Step& st : steps) {
            for (hipEvent_t e : {st.t0, st.ev})
                if (e) (void)hipEventDestroy(e);
            if (st.h_dig) (void)hipHostFree(st.h_dig);
            if (st.h_act) (void)hipHostFree(st.h_act);
            if (st.h_ol) (void)hipHostFree(st.h_ol);
        }
        if (ring) (void)hipFree(ring);
        if (d_chains) (void)hipFree(d_chains);
        if (h_chains) (void)hipHostFree(h_chains);
        if (d_dig) (void)hipFree(d_dig);
        if (d_act) (void)hipFree(d_act);
        if (d_ol) (void)hipFree(d_ol);
        if (hstream) (void)hipStreamDestroy(hstream);
        if (copy) (void)hipStreamDestroy(copy);
        if (stream) (void)hipStreamDestroy(stream);
    }
    uint8_t* get_block() {  // pool_mu not held: new pinned blocks are allocated outside it
        {
            std::lock_guard<std::mutex> lk(pool_mu);
            if (!pool.empty()) {
                uint8_t* b = pool.back();
                pool.pop_back();
                return b;
            }
        }
        // a slab of kSlabBlocks at once: a hipHostMalloc costs milliseconds under load, and the
        // staging peak grows in steps of many blocks when many writers are open
        pool_misses++;
        void* p = nullptr;
        Guard g(device);
        if (hipHostMalloc(&p, kSlabBlocks * kBlock, hipHostMallocDefault) != hipSuccess) return nullptr;
        uint8_t* s = static_cast<uint8_t*>(p);
        std::lock_guard<std::mutex> lk(pool_mu);
        slabs.push_back(s);
        for (size_t i = 1; i < kSlabBlocks; i++) pool.push_back(s + i * kBlock);
        return s;
    }
    void loop();
};

// The batcher's lifetime state, shared by the batcher and every writer it opened (refcounted): a
// writer call that starts while or after kcdc_bw_batcher_free runs sees `closing` here -- memory
// that outlives the batcher -- and returns KCDC_EINVAL without touching the freed device state.
struct BwCtl {
    std::atomic<int> inside{0};        // threads inside a writer call (batcher_free waits for them)
    std::atomic<bool> closing{false};  // kcdc_bw_batcher_free has started
    std::atomic<bool> detached{false}; // ... and has detached every open writer (w->b = null)
};

struct kcdc_bw_batcher {
    const Algo* algo = nullptr;
    std::vector<BwDev*> devs;
    std::mutex mu;                   // writer assignment
    std::shared_ptr<BwCtl> ctl = std::make_shared<BwCtl>();
};

struct kcdc_bw {
    BwDev* b = nullptr;              // the device batcher this writer ships through (null once freed)
    std::shared_ptr<BwCtl> ctl;      // the batcher's lifetime state (outlives the batcher)
    int device = 0;                  // HIP device of the arenas
    uint64_t hint = 0;               // expected object size (0: unknown)
    uint64_t counted = 0;            // this writer's share of b->load
    std::mutex mu;               // staging (the writer's thread vs the round thread's collection)
    std::condition_variable cv;  // write(): bytes were shipped
    std::vector<Blk> blocks;     // unshipped bytes [shipped, written); only the last may be partial
    uint64_t written = 0;        // (mu)
    uint64_t shipped = 0;        // bytes handed to a round (mu)
    bool finishing = false;      // (mu)
    // round thread (and batcher mu for what writers read):
    uint8_t* arena = nullptr;    // device: stream byte p at arena + (p - origin)
    uint8_t* spare = nullptr;    // the other arena: compaction copies the live bytes over and swaps
    uint64_t origin = 0;
    uint64_t tail_pos = 0;       // first byte the next region needs (last final cut - 64)
    uint64_t launched_to = 0;    // end of the last completed region (the chunk in progress was tested up to it)
    uint64_t frontier = 0;       // last final cut (0: none yet)
    bool final_sent = false;     // the finishing region is issued
    std::vector<uint64_t> ready; // final cuts not taken yet (batcher mu)
    size_t ready_head = 0;
    // cuts ever pushed to / taken from `ready` (written under the batcher mu): kcdc_bw_cuts returns
    // without that mutex when they are equal, so polling writers do not contend with the round thread
    std::atomic<uint64_t> ready_pushed{0}, ready_taken{0};
    bool done = false;           // (batcher mu)
    uint64_t fixed_next = 0;     // FIXED names: the next cut (no data is read)
    // content IDs (batcher mu): entry wseq = ids_base + i, in cut order; taken as a ready prefix
    struct IdEntry {
        uint64_t cut;
        bool ready;
        uint8_t id[32];
    };
    std::deque<IdEntry> ids;
    uint64_t ids_base = 0;       // wseq of ids.front()
    uint64_t ids_made = 0;       // entries ever created
    uint64_t ids_ready = 0;      // entries whose digest has arrived
    // entries ready at the front / taken (kcdc_bw_cuts_ids answers "nothing new" without the mutex)
    std::atomic<uint64_t> ids_pub{0}, ids_taken{0};
    uint64_t id_from = 0;        // start of the next final chunk
};

namespace {
struct SrcPiece {
    const uint8_t* src;
    uint64_t pos, len;  // stream position of the first byte
};
struct Job {
    kcdc_bw* w;
    uint64_t to;  // region end (shipped after this round)
    bool finishing;
    std::vector<SrcPiece> pcs;
    std::vector<uint8_t*> retire;  // blocks fully shipped by this round (free after its gather)
};
struct Round {
    int m = 0;  // meta set
    std::vector<Job> jobs;
    uint32_t n = 0;
    std::vector<uint64_t> cbase;
    uint64_t fresh = 0;
    bool live = false;
    bool recycled = false;  // its retired blocks are back in the pool
};
}  // namespace

void BwDev::loop() {
    Guard g(device);
    Round inflight;
    int next_meta = 0;
    // Wait for round r's cuts and apply them (final cuts, frontier, tail position).  mu not held.
    auto complete = [&](Round& r) -> int {
        if (!r.live) return KCDC_OK;
        r.live = false;
        Meta& M = meta[r.m];
        const auto t0 = std::chrono::steady_clock::now();
        hipError_t e = hipEventSynchronize(M.done);
        t_wait += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (e != hipSuccess) return hip_err(e, "writer round");
        float gms = 0, kms = 0, a = 0, z = 0;
        if (hipEventElapsedTime(&gms, M.g0, M.gathered) == hipSuccess) {
            t_gather += gms * 1e-3;
            if (hipEventElapsedTime(&a, ev_ref, M.g0) == hipSuccess) busy.emplace_back(a, a + gms);
        }
        if (r.n && hipEventElapsedTime(&kms, M.k0, M.done) == hipSuccess) {
            t_kernel += kms * 1e-3;
            if (hipEventElapsedTime(&z, ev_ref, M.k0) == hipSuccess) busy.emplace_back(z, z + kms);
        }
        const uint32_t n = r.n;
        const uint64_t* hp = M.h;
        const auto l0 = std::chrono::steady_clock::now();
        std::lock_guard<std::mutex> lk(mu);
        t_lock += std::chrono::duration<double>(std::chrono::steady_clock::now() - l0).count();
        // after an error a writer of this round may already be freed (kcdc_bw_free does not wait
        // for rounds then): touch none of them
        if (error) return error;
        shipped_bytes += r.fresh;
        for (uint32_t k = 0; k < n; k++) {
            Job& j = r.jobs[k];
            kcdc_bw* w = j.w;
            if (!j.retire.empty()) {
                std::lock_guard<std::mutex> pl(pool_mu);
                for (uint8_t* blk : j.retire) pool.push_back(blk);
            }
            const uint64_t len = j.to - w->tail_pos;
            const uint64_t cnt = hp[5 * n + k];
            if (cnt == ~0ull || cnt > len / algo->min_size() + 2)
                return set_error(KCDC_EIO, "writer round: the device lost a stream");
            const uint64_t* c = hp + 6 * n + r.cbase[k];
            const uint64_t fin = j.finishing ? cnt : (cnt ? cnt - 1 : 0);
            if (ids.on) {  // every final chunk [id_from, cut) gets an ID entry and, in id_create, a chain
                for (uint64_t t = 0; t < fin; t++) {
                    const uint64_t cut = w->tail_pos + c[t];
                    w->ids.push_back(kcdc_bw::IdEntry{cut, false, {}});
                    newc.push_back(NewChunk{w, w->ids_made++, w->id_from, cut - w->id_from});
                    w->id_from = cut;
                }
            } else {
                for (uint64_t t = 0; t < fin; t++) w->ready.push_back(w->tail_pos + c[t]);
                w->ready_pushed.fetch_add(fin, std::memory_order_release);
            }
            if (fin) w->frontier = w->tail_pos + c[fin - 1];
            w->launched_to = j.to;
            w->tail_pos = w->frontier >= kHist ? w->frontier - kHist : 0;
            if (j.finishing) w->done = true;
        }
        cv_done.notify_all();
        return KCDC_OK;
    };

    // The round in flight's pinned blocks go back to the pool once its gather has copied them (the
    // split reads the arenas), not when its cuts arrive.  mu held.
    auto recycle = [&](Round& r) {
        if (!r.live || r.recycled || hipEventQuery(meta[r.m].gathered) != hipSuccess) return;
        std::lock_guard<std::mutex> pl(pool_mu);
        for (Job& j : r.jobs) {
            for (uint8_t* blk : j.retire) pool.push_back(blk);
            j.retire.clear();
        }
        r.recycled = true;
    };
    std::unique_lock<std::mutex> lk(mu);
    auto last = std::chrono::steady_clock::now();
    for (;;) {
        auto work = [&] {
            return stop || error || staged.load() >= round_bytes || capped.load() > 0 || finish_pending.load() > 0;
        };
        // Ship when a round's worth is staged, a writer is blocked on its cap or finishing, or
        // max_wait after the first unshipped byte (or after the last round).  Meanwhile apply
        // the round in flight as soon as the device has finished it (its writers may be waiting
        // for cuts) -- but do not block on it: the next round's gather should start while it splits.
        bool timed_out = false;
        const auto idle0 = std::chrono::steady_clock::now();
        while (!work() && !timed_out) {
            recycle(inflight);
            if (inflight.live) {
                if (hipEventQuery(meta[inflight.m].done) == hipSuccess) {
                    lk.unlock();
                    int rc = complete(inflight);
                    if (rc == KCDC_OK && ids.on) rc = id_create();
                    lk.lock();
                    if (rc != KCDC_OK) {
                        lk.unlock();
                        fail(rc);
                        lk.lock();
                    }
                } else {
                    cv_round.wait_for(lk, std::chrono::microseconds(100), work);
                }
                continue;
            }
            if (staged.load() > 0) {
                const auto since_tp = std::chrono::steady_clock::time_point(std::chrono::nanoseconds(since.load()));
                const auto due = std::max(last, since_tp) + wait;
                if (cv_round.wait_until(lk, due, work)) break;
                timed_out = std::chrono::steady_clock::now() >= due;
            } else {
                // bounded: writers change `staged`, `capped` and `finish_pending` without this
                // mutex, so a notify can land between the predicate check and the wait
                cv_round.wait_for(lk, std::chrono::milliseconds(1), [&] { return work() || staged.load() > 0; });
            }
        }
        t_idle += std::chrono::duration<double>(std::chrono::steady_clock::now() - idle0).count();
        if (error) break;
        if (staged.load() == 0 && finish_pending.load() == 0) {
            if (stop) break;
            continue;
        }
        recycle(inflight);
        // ---- collect round R: every writer's staged bytes (writers keep writing meanwhile)
        const auto t0 = std::chrono::steady_clock::now();
        writer_refs++;  // until R is issued (unref_writers below)
        Round R;
        R.m = next_meta;
        struct Move {
            uint8_t* dst;
            const uint8_t* src;
            uint64_t len;
        };
        std::vector<Move> compact;
        bool overflow = false;
        for (kcdc_bw* w : open) {
            if (w->done || w->final_sent) continue;
            std::lock_guard<std::mutex> wl(w->mu);
            const uint64_t to = w->written;
            if (to == w->shipped && !w->finishing) continue;
            Job j{w, to, w->finishing, {}, {}};
            for (size_t i = 0; i < w->blocks.size(); i++) {
                Blk& bk = w->blocks[i];
                if (bk.end > bk.start) j.pcs.push_back(SrcPiece{bk.p + bk.start, bk.pos, bk.end - bk.start});
                bk.pos += bk.end - bk.start;
                bk.start = bk.end;
                if (bk.end == kBlock || i + 1 < w->blocks.size()) j.retire.push_back(bk.p);
            }
            if (!w->blocks.empty() && w->blocks.back().end < kBlock) {  // the writer keeps filling it
                const Blk keep = w->blocks.back();
                w->blocks.assign(1, keep);
            } else {
                w->blocks.clear();
            }
            staged -= to - w->shipped;
            R.fresh += to - w->shipped;
            w->shipped = to;
            w->cv.notify_all();
            if (w->finishing) {
                w->final_sent = true;
                finish_pending--;
            }
            if (to - w->origin > arena_cap) {
                // compact: the live bytes [tail_pos, shipped before this round) -- a superset of what
                // the round in flight will leave -- to the spare arena (congruent mod 16), queued on
                // the copy stream after the in-flight gather; the round in flight keeps reading the
                // old arena, so nothing waits for it
                const uint64_t from = w->tail_pos, norigin = from & ~uint64_t(15);
                const uint64_t have = j.pcs.empty() ? to - from : j.pcs.front().pos - from;
                compact.push_back({w->spare + (from - norigin), w->arena + (from - w->origin), have});
                std::swap(w->arena, w->spare);
                w->origin = norigin;
                if (to - w->origin > arena_cap) overflow = true;
            }
            R.jobs.push_back(std::move(j));
        }
        rounds++;
        lk.unlock();
        auto lap = [&, tp = std::chrono::steady_clock::now()](int i) mutable {
            const auto t = std::chrono::steady_clock::now();
            t_seg[i] += std::chrono::duration<double>(t - tp).count();
            tp = t;
        };
        t_seg[0] += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        int rc = overflow ? set_error(KCDC_EIO, "writer arena overflow") : KCDC_OK;
        if (rc == KCDC_OK && ids.on && !compact.empty()) {  // the ring copies may still read these arenas
            hipError_t e = hipStreamWaitEvent(copy, copy_ev, 0);
            if (e != hipSuccess) rc = hip_err(e, "writer compaction wait");
        }
        // Compactions: one copy launch for all of them (one hipMemcpyAsync each was a blit kernel
        // each), before the gather; their pieces lead the round's piece list.  The ring copies of
        // the content IDs wait for them (compacted_ev), not for the gather.
        std::vector<Piece> pieces;
        uint64_t tasks = 0, ctasks = 0;
        for (const Move& mv : compact) {
            if (!mv.len) continue;
            pieces.push_back(Piece{mv.src, mv.dst, mv.len, ctasks});
            ctasks += (mv.len + kTask - 1) / kTask;
        }
        const size_t ncp = pieces.size();
        for (Job& j : R.jobs) {
            for (const SrcPiece& sp : j.pcs) {
                pieces.push_back(Piece{sp.src, j.w->arena + (sp.pos - j.w->origin), sp.len, tasks});
                tasks += (sp.len + kTask - 1) / kTask;
            }
        }
        Meta& M = meta[R.m];
        lap(1);
        if (rc == KCDC_OK && M.pcap < pieces.size()) {
            if (M.dp) (void)hipFree(M.dp);
            if (M.hp) (void)hipHostFree(M.hp);
            M.dp = M.hp = nullptr;
            M.pcap = 0;
            const size_t want = std::max<size_t>(pieces.size() * 2, 1024);
            hipError_t e = hipMalloc(&M.dp, want * sizeof(Piece));
            if (e == hipSuccess) e = hipHostMalloc(&M.hp, want * sizeof(Piece), hipHostMallocDefault);
            if (e != hipSuccess) rc = hip_err(e, "writer gather list");
            else M.pcap = want;
        }
        if (rc == KCDC_OK) {
            hipError_t e = hipEventRecord(M.g0, copy);
            if (e == hipSuccess && !pieces.empty()) {
                std::memcpy(M.hp, pieces.data(), pieces.size() * sizeof(Piece));
                e = hipMemcpyAsync(M.dp, M.hp, pieces.size() * sizeof(Piece), hipMemcpyHostToDevice, copy);
                if (e == hipSuccess && ncp) {
                    const unsigned grid = static_cast<unsigned>(std::min<uint64_t>(ctasks, 2 * kGatherWGs));
                    hipLaunchKernelGGL(bw_gather_kernel, dim3(grid), dim3(256), 0, copy, M.dp, static_cast<uint32_t>(ncp),
                                       ctasks);
                    e = hipGetLastError();
                }
            }
            if (e == hipSuccess && ids.on) e = hipEventRecord(compacted_ev, copy);
            if (e == hipSuccess && pieces.size() > ncp) {
                const unsigned grid = static_cast<unsigned>(std::min<uint64_t>(tasks, kGatherWGs));
                hipLaunchKernelGGL(bw_gather_kernel, dim3(grid), dim3(256), 0, copy, M.dp + ncp,
                                   static_cast<uint32_t>(pieces.size() - ncp), tasks);
                e = hipGetLastError();
            }
            if (e == hipSuccess) e = hipEventRecord(M.gathered, copy);
            if (e != hipSuccess) rc = hip_err(e, "writer gather");
        }
        lap(2);
        // round k's cuts are round k+1's chunk starts
        if (rc == KCDC_OK && inflight.live) {
            rc = complete(inflight);
            // its final chunks' ring copies queue on the copy stream behind this round's compactions
            if (rc == KCDC_OK && ids.on) rc = id_create();
        }
        lap(3);
        // ---- launch R over every job's region [tail_pos, to)
        if (rc == KCDC_OK) {
            const uint32_t n = static_cast<uint32_t>(R.jobs.size());
            R.n = n;
            R.cbase.resize(n);
            uint64_t cuts_cap = 0;
            for (uint32_t k = 0; k < n; k++) {
                R.cbase[k] = cuts_cap;
                cuts_cap += (R.jobs[k].to - R.jobs[k].w->tail_pos) / algo->min_size() + 2;
            }
            const size_t words = 6ull * n + cuts_cap + 1;
            if (M.cap < words) {
                if (M.d) (void)hipFree(M.d);
                if (M.h) (void)hipHostFree(M.h);
                M.d = M.h = nullptr;
                M.cap = 0;
                const size_t want = std::max<size_t>(words * 2, 1u << 16);
                hipError_t e = hipMalloc(&M.d, want * 8);
                if (e == hipSuccess) e = hipHostMalloc(&M.h, want * 8, hipHostMallocDefault);
                if (e != hipSuccess) rc = hip_err(e, "writer metadata");
                else M.cap = want;
            }
            if (rc == KCDC_OK && n) {
                uint64_t* hp = M.h;
                for (uint32_t k = 0; k < n; k++) {
                    kcdc_bw* w = R.jobs[k].w;
                    hp[k] = reinterpret_cast<uint64_t>(w->arena + (w->tail_pos - w->origin));  // ptrs
                    hp[n + k] = R.jobs[k].to - w->tail_pos;                                      // lens
                    hp[2 * n + k] = w->frontier - w->tail_pos;                                   // starts
                    hp[3 * n + k] = R.cbase[k];                                                  // cut_base
                    // the chunk in progress was tested up to the last completed region's end; its
                    // last byte is tested again: a candidate there cut the region at its end, and
                    // complete() cannot tell that cut from the region end, so it was not taken
                    hp[4 * n + k] = w->launched_to > w->tail_pos + 1 ? w->launched_to - w->tail_pos - 1 : 0;  // resume
                }
                uint64_t* dp = M.d;
                hipError_t e = hipStreamWaitEvent(stream, M.gathered, 0);
                if (e == hipSuccess) e = hipEventRecord(M.k0, stream);
                if (e == hipSuccess) e = hipMemcpyAsync(dp, hp, 5ull * n * 8, hipMemcpyHostToDevice, stream);
                if (e != hipSuccess) rc = hip_err(e, "writer metadata H2D");
                if (rc == KCDC_OK) {
                    SplitArgs s;
                    s.ptrs = reinterpret_cast<const uint8_t* const*>(dp);
                    s.lens = dp + n;
                    s.starts = dp + 2 * n;
                    s.cut_base = dp + 3 * n;
                    s.resume = dp + 4 * n;
                    s.counts = dp + 5 * n;
                    s.cuts = dp + 6 * n;
                    s.cuts_cap = cuts_cap;
                    s.nstreams = n;
                    rc = launch_split_batch(*algo, s, device, stream);
                }
                if (rc == KCDC_OK) {
                    e = hipMemcpyAsync(hp + 5 * n, dp + 5 * n, (n + cuts_cap) * 8, hipMemcpyDeviceToHost, stream);
                    if (e == hipSuccess) e = hipEventRecord(M.done, stream);
                    if (e != hipSuccess) rc = hip_err(e, "writer cuts D2H");
                }
            } else if (rc == KCDC_OK) {
                hipError_t e = hipEventRecord(M.done, copy);
                if (e != hipSuccess) rc = hip_err(e, "writer round event");
            }
        }
        lap(4);
        t_submit += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        last = std::chrono::steady_clock::now();
        if (rc != KCDC_OK) {
            fail(rc);
            lk.lock();
            unref_writers();
            break;
        }
        R.live = true;
        inflight = std::move(R);
        next_meta ^= 1;
        lk.lock();
        unref_writers();
    }
    lk.unlock();
    if (inflight.live && !error) {
        int rc = complete(inflight);
        if (rc == KCDC_OK && ids.on) rc = id_create();
        if (rc != KCDC_OK) fail(rc);
    }
    lk.lock();
    cv_done.notify_all();
    if (ids.on) {  // the hash thread names the chains of the last rounds, then ends
        hstop = true;
        cv_hash.notify_all();
        lk.unlock();
        if (hth.joinable()) hth.join();
        lk.lock();
        cv_done.notify_all();
    }
}

void BwDev::fail(int rc) {
    std::lock_guard<std::mutex> lk(mu);
    if (!error) {
        errmsg = kcdc_last_error();
        error = rc;
    }
    cv_done.notify_all();
    cv_space.notify_all();
    cv_hash.notify_all();
    for (kcdc_bw* w : open) {
        std::lock_guard<std::mutex> wl(w->mu);
        w->cv.notify_all();
    }
}

// ---------------------------------------------------------------- content IDs
int BwDev::ids_enable(const char* name, const uint8_t* key, uint32_t key_len) {
    uint32_t out = 0;
    const int kind = hash_chain_kind(name, &out);
    if (kind < 0) return kind;
    if (key_len && !key) return set_error(KCDC_EINVAL, "null key");
    ids.name = name;
    ids.key.assign(key, key + key_len);
    ids.out = out;
    ids.kind = kind;
    // slices of 256 KiB per chain per step: a 4 MiB chunk is named after ~16 steps
    step_blocks = kind == 1 ? 2048 : 4096;
    // chains in flight set the naming rate (one chain: ~50 MB/s of BLAKE2b), so the ring holds 64
    // rounds: 16 GiB, ~3,000 chunks of 4-5 MiB at the default 256 MiB rounds (of 288 GB of HBM)
    ring_cap = std::max<uint64_t>(64 * round_bytes, 1ull << 30);
    if (test_id_ring_bytes()) ring_cap = std::max<uint64_t>(test_id_ring_bytes(), 16) & ~uint64_t(15);  // tests: wrap and backpressure
    chain_cap = 16384;
    Guard g(device);
    hipError_t e = hipStreamCreateWithFlags(&hstream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&idcopy, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&compacted_ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(compacted_ev, copy);
    if (e == hipSuccess) e = hipMalloc(&ring, ring_cap);
    if (e == hipSuccess) e = hipMalloc(&d_chains, sizeof(HashChain) * chain_cap);
    if (e == hipSuccess) e = hipHostMalloc(&h_chains, sizeof(HashChain) * chain_cap, hipHostMallocDefault);
    if (e == hipSuccess) e = hipMalloc(&d_dig, 32ull * chain_cap);
    if (e == hipSuccess) e = hipMalloc(&d_act, 4ull * chain_cap);
    if (e == hipSuccess) e = hipMalloc(&d_ol, 16ull * chain_cap);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&copy_ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(copy_ev, idcopy);
    for (hipEvent_t& ev : pub_ev)
        if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipHostMalloc(&h_rp, sizeof(Piece) * kPubEv * kPubPieces, hipHostMallocDefault);
    if (e == hipSuccess) e = hipMalloc(&d_rp, sizeof(Piece) * kPubEv * kPubPieces);
    for (Step& st : steps) {
        if (e == hipSuccess) e = hipHostMalloc(&st.h_dig, 32ull * chain_cap, hipHostMallocDefault);
        if (e == hipSuccess) e = hipHostMalloc(&st.h_act, 4ull * chain_cap, hipHostMallocDefault);
        if (e == hipSuccess) e = hipHostMalloc(&st.h_ol, 16ull * chain_cap, hipHostMallocDefault);
        if (e == hipSuccess) e = hipEventCreate(&st.t0);
        if (e == hipSuccess) e = hipEventCreate(&st.ev);
    }
    if (e != hipSuccess) return hip_err(e, "writer content IDs: device memory");
    ids.on = true;
    hth = std::thread([this] { hash_loop(); });
    return KCDC_OK;
}

// Undo ids_enable on a device whose batcher could not enable content IDs on every device (no writer
// has opened, so no chain exists): stop the hash thread, free what ids_enable allocated.
void BwDev::ids_disable() {
    if (hth.joinable()) {
        {
            std::lock_guard<std::mutex> lk(mu);
            hstop = true;
        }
        cv_hash.notify_all();
        hth.join();
    }
    Guard g(device);
    for (hipEvent_t* ev : {&compacted_ev, &copy_ev})
        if (*ev) (void)hipEventDestroy(*ev), *ev = nullptr;
    for (hipEvent_t& ev : pub_ev)
        if (ev) (void)hipEventDestroy(ev), ev = nullptr;
    for (Step& st : steps) {
        for (hipEvent_t* ev : {&st.t0, &st.ev})
            if (*ev) (void)hipEventDestroy(*ev), *ev = nullptr;
        for (void** p : {reinterpret_cast<void**>(&st.h_dig), reinterpret_cast<void**>(&st.h_act),
                         reinterpret_cast<void**>(&st.h_ol)})
            if (*p) (void)hipHostFree(*p), *p = nullptr;
    }
    for (void** p : {reinterpret_cast<void**>(&h_rp), reinterpret_cast<void**>(&h_chains)})
        if (*p) (void)hipHostFree(*p), *p = nullptr;
    for (void** p : {reinterpret_cast<void**>(&d_rp), reinterpret_cast<void**>(&ring), reinterpret_cast<void**>(&d_chains),
                     reinterpret_cast<void**>(&d_dig), reinterpret_cast<void**>(&d_act), reinterpret_cast<void**>(&d_ol)})
        if (*p) (void)hipFree(*p), *p = nullptr;
    for (hipStream_t* st : {&hstream, &idcopy})
        if (*st) (void)hipStreamDestroy(*st), *st = nullptr;
    std::lock_guard<std::mutex> lk(mu);
    ids = IdCfg{};
    hstop = false;
}

// The last completed round's final chunks (newc) become chains: ring space and a slot each, a
// copy from the writer's arena into the ring, then (after an event on the copy stream) the chain
// is published to the hash thread.  Called right after complete(): the arena pointers are those of
// the compactions of the last collected round, and the copies (idcopy stream) wait for those
// (compacted_ev); any later compaction waits for the copies (copy_ev).  When the ring is full it publishes what it has copied and waits for the
// hash thread to free space.
int BwDev::id_create() {
    std::vector<NewChunk> work;
    {
        std::lock_guard<std::mutex> lk(mu);
        if (error) {  // a writer of these chunks may already be freed (kcdc_bw_free after an error)
            newc.clear();
            return error;
        }
        if (newc.empty()) return KCDC_OK;
        work.swap(newc);
        writer_refs++;  // the arenas read below stay allocated until this returns
    }
    struct Unref {
        BwDev* b;
        ~Unref() {
            std::lock_guard<std::mutex> lk(b->mu);
            b->unref_writers();
        }
    } unref{this};
    Guard g(device);
    {
        const hipError_t e = hipStreamWaitEvent(idcopy, compacted_ev, 0);
        if (e != hipSuccess) return hip_err(e, "writer content IDs: compaction wait");
    }
    std::vector<Chain> made;
    std::vector<Piece> pcs;  // the made chains' ring copies (to 16-byte aligned ring slots)
    uint64_t ptasks = 0;
    auto publish = [&]() -> int {
        if (made.empty()) return KCDC_OK;
        uint64_t seq;
        {
            std::lock_guard<std::mutex> lk(mu);
            if (error) {  // no copies for chains that will never be named
                made.clear();
                pcs.clear();
                return error;
            }
            seq = pub_seq;
        }
        // the slot of publish seq - kPubEv (event, pinned pieces) must be complete before reuse
        hipError_t e = hipSuccess;
        if (seq >= kPubEv) e = hipEventSynchronize(pub_ev[seq % kPubEv]);
        if (e == hipSuccess && !pcs.empty()) {  // one copy launch for the whole publish
            Piece* hp = h_rp + (seq % kPubEv) * kPubPieces;
            Piece* dp = d_rp + (seq % kPubEv) * kPubPieces;
            std::memcpy(hp, pcs.data(), pcs.size() * sizeof(Piece));
            e = hipMemcpyAsync(dp, hp, pcs.size() * sizeof(Piece), hipMemcpyHostToDevice, idcopy);
            if (e == hipSuccess) {
                const unsigned grid = static_cast<unsigned>(std::min<uint64_t>(ptasks, 2 * kGatherWGs));
                hipLaunchKernelGGL(bw_realign_kernel, dim3(grid), dim3(256), 0, idcopy, dp,
                                   static_cast<uint32_t>(pcs.size()), ptasks);
                e = hipGetLastError();
            }
        }
        pcs.clear();
        ptasks = 0;
        if (e == hipSuccess) e = hipEventRecord(pub_ev[seq % kPubEv], idcopy);
        if (e == hipSuccess) e = hipEventRecord(copy_ev, idcopy);  // (later compactions wait on it)
        if (e != hipSuccess) return hip_err(e, "writer content IDs: copy event");
        {
            std::lock_guard<std::mutex> lk(mu);
            pub_seq = seq + 1;
            for (Chain& c : made) {
                c.pub = seq;
                chains.push_back(c);
            }
            chain_head += made.size();
            undone += made.size();
            id_chains += made.size();
        }
        made.clear();
        cv_hash.notify_one();
        return KCDC_OK;
    };
    for (const NewChunk& nc : work) {
        const uint64_t need = (nc.len + 15) & ~uint64_t(15);
        if (need > ring_cap) return set_error(KCDC_EIO, "writer content IDs: chunk larger than the ID ring");
        const uint8_t* src = nc.w->arena + (nc.pos - nc.w->origin);
        uint64_t at = 0;
        if (made.size() >= kPubPieces) {
            const int rc = publish();
            if (rc != KCDC_OK) return rc;
        }
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu);
                if (error) return error;
                if (chain_tail == chain_head && made.empty()) {
                    // the ring is empty: restart at a ring boundary, so a chunk larger than what is
                    // left before the wrap does not wait for space nothing will free
                    ring_head = ring_tail = (ring_head + ring_cap - 1) / ring_cap * ring_cap;
                }
                at = ring_head;  // (a multiple of 16)
                if (at % ring_cap + need > ring_cap) at += ring_cap - at % ring_cap;  // no chunk wraps
                if (at + need - ring_tail <= ring_cap && chain_head + made.size() - chain_tail < chain_cap) break;
                if (made.empty()) {
                    if (chain_tail == chain_head)
                        return set_error(KCDC_EIO, "writer content IDs: ring full with no chain in flight");
                    const auto w0 = std::chrono::steady_clock::now();
                    cv_space.wait_for(lk, std::chrono::milliseconds(2));
                    t_space += std::chrono::duration<double>(std::chrono::steady_clock::now() - w0).count();
                    continue;
                }
            }
            const int rc = publish();  // the waiting chains may need the bytes just copied
            if (rc != KCDC_OK) return rc;
        }
        const uint64_t cn = chain_head + made.size();  // (only this thread grows chain_head)
        const uint32_t slot = static_cast<uint32_t>(cn % chain_cap);
        uint8_t* dst = ring + at % ring_cap;
        if (nc.len) {
            pcs.push_back(Piece{src, dst, nc.len, ptasks});
            ptasks += (nc.len + kTask - 1) / kTask;
        }
        HashChain& hc = h_chains[slot];
        std::memset(&hc, 0, sizeof(hc));
        hc.src = reinterpret_cast<uint64_t>(dst);
        hc.len = nc.len;
        hc.next = ~0ull;
        hc.out = slot;
        const uint64_t bb = ids.kind == 2 ? 64 : 128;
        const uint64_t nblk = ids.kind == 3 ? 1 : nc.len ? (nc.len + bb - 1) / bb : 1;
        made.push_back(Chain{nc.w, nc.wseq, at, at + need, nc.len, nblk, 0, false});
        ring_head = at + need;
    }
    return publish();
}

// Issue one step over every published chain with blocks left (issued = false: none).
int BwDev::id_issue(Step& st, bool& issued) {
    issued = false;
    uint32_t n = 0;
    st.done.clear();
    {
        std::lock_guard<std::mutex> lk(mu);
        if (undone == 0) return KCDC_OK;
        while (pub_done < pub_seq && hipEventQuery(pub_ev[pub_done % kPubEv]) == hipSuccess) pub_done++;
        for (uint64_t k = 0; k < chains.size(); k++) {
            Chain& c = chains[k];
            if (c.fin || c.done >= c.nblk) continue;
            if (c.pub >= pub_done) break;  // its ring copy (and every later chain's) is not done yet
            const uint64_t cn = chain_tail + k;
            if (ids.kind == 3) {  // whole chunks, in this step's order
                st.h_ol[n] = c.ring_at % ring_cap;
                st.h_ol[chain_cap + n] = c.len;
                c.done = c.nblk;
                st.done.emplace_back(cn, n);
            } else {  // (a chain's first step takes its record from h_chains)
                st.h_act[n] = static_cast<uint32_t>(cn % chain_cap) | (c.done == 0 ? kChainNew : 0u);
                c.done = std::min(c.nblk, c.done + step_blocks);
                if (c.done == c.nblk) st.done.emplace_back(cn, static_cast<uint32_t>(cn % chain_cap));
            }
            if (c.done == c.nblk) undone--;
            n++;
        }
        chain_steps += n;
    }
    if (n == 0) return KCDC_OK;
    // the BLAKE2 kinds read new chains' records, the active list and their digests through
    // host-mapped memory (one launch, no copies); kind 3 hashes whole chunks from the step's list
    hipError_t e = hipEventRecord(st.t0, hstream);
    if (e != hipSuccess) return hip_err(e, "writer content IDs: chain upload");
    int rc = KCDC_OK;
    if (ids.kind == 3) {
        e = hipMemcpyAsync(d_ol, st.h_ol, 8ull * n, hipMemcpyHostToDevice, hstream);
        if (e == hipSuccess) e = hipMemcpyAsync(d_ol + chain_cap, st.h_ol + chain_cap, 8ull * n, hipMemcpyHostToDevice, hstream);
        if (e != hipSuccess) return hip_err(e, "writer content IDs: chunk list");
        rc = kcdc_hash_chunks_device(ids.name.c_str(), ring, d_ol, d_ol + chain_cap, nullptr, n, ids.key.data(),
                                     static_cast<uint32_t>(ids.key.size()), d_dig, 32, hstream);
        if (rc == KCDC_OK) e = hipMemcpyAsync(st.h_dig, d_dig, 32ull * n, hipMemcpyDeviceToHost, hstream);
    } else {
        rc = launch_hash_chains(ids.name.c_str(), ids.key.data(), static_cast<uint32_t>(ids.key.size()), d_chains,
                                h_chains, st.h_act, n, step_blocks, st.h_dig, 32, hstream);
    }
    if (rc != KCDC_OK) return rc;
    if (e == hipSuccess) e = hipEventRecord(st.ev, hstream);
    if (e != hipSuccess) return hip_err(e, "writer content IDs: hash step");
    issued = true;
    return KCDC_OK;
}

// Wait for a step, then hand its finished digests to their writers and free the ring's head.
int BwDev::id_deliver(Step& st) {
    // polled with sleeps: a hash thread parked in hipEventSynchronize for a 5 ms step held up the
    // round thread's HIP calls (its round waits doubled and the device idled half the time)
    hipError_t q;
    while ((q = hipEventQuery(st.ev)) == hipErrorNotReady) std::this_thread::sleep_for(std::chrono::microseconds(200));
    if (q != hipSuccess) return hip_err(q, "writer content IDs: hash step");
    float ms = 0;
    const bool timed = hipEventElapsedTime(&ms, st.t0, st.ev) == hipSuccess;
    std::lock_guard<std::mutex> lk(mu);
    if (timed) t_hash += ms * 1e-3;
    id_steps++;
    for (const auto& d : st.done) {
        Chain& c = chains[d.first - chain_tail];
        c.fin = true;
        if (!c.w) continue;  // its writer was freed
        kcdc_bw::IdEntry& en = c.w->ids[c.wseq - c.w->ids_base];
        std::memcpy(en.id, st.h_dig + 32ull * d.second, ids.out);
        en.ready = true;
        c.w->ids_ready++;
    }
    // publish each touched writer's ready prefix (digests arrive out of order across chains)
    for (const auto& d : st.done) {
        Chain& c = chains[d.first - chain_tail];
        if (!c.w) continue;
        kcdc_bw* w = c.w;
        uint64_t k = w->ids_pub.load(std::memory_order_relaxed);
        while (k - w->ids_base < w->ids.size() && w->ids[k - w->ids_base].ready) k++;
        w->ids_pub.store(k, std::memory_order_release);
    }
    st.done.clear();
    bool freed = false;
    while (!chains.empty() && chains.front().fin) {
        ring_tail = chains.front().ring_end;
        chains.pop_front();
        chain_tail++;
        freed = true;
    }
    cv_done.notify_all();
    if (freed) cv_space.notify_all();
    return KCDC_OK;
}

// The hash thread: keep two steps in flight while chains have blocks left; end once the round
// thread has stopped and every chain is named (or on an error).
void BwDev::hash_loop() {
    Guard g(device);
    std::deque<int> live;  // steps in flight, in issue order
    int next = 0;
    for (;;) {
        int rc = KCDC_OK;
        while (rc == KCDC_OK && live.size() < 2) {
            bool issued = false;
            rc = id_issue(steps[next], issued);
            if (!issued) break;
            live.push_back(next);
            next ^= 1;
        }
        if (rc == KCDC_OK && !live.empty()) {
            rc = id_deliver(steps[live.front()]);
            live.pop_front();
        }
        if (rc != KCDC_OK) {
            fail(rc);
            break;
        }
        if (!live.empty()) continue;
        std::unique_lock<std::mutex> lk(mu);
        if (error || (hstop && chain_tail == chain_head)) break;
        const auto w0 = std::chrono::steady_clock::now();
        if (undone == 0)
            cv_hash.wait_for(lk, std::chrono::milliseconds(5), [&] { return error || hstop || undone > 0; });
        else  // chains waiting for their ring copies
            cv_hash.wait_for(lk, std::chrono::microseconds(200));
        t_hidle += std::chrono::duration<double>(std::chrono::steady_clock::now() - w0).count();
    }
    for (int i : live) (void)hipEventSynchronize(steps[i].ev);  // (after an error: nothing reads the buffers after this)
}

uint64_t& kcdc::test_id_ring_bytes() {
    static uint64_t v = 0;
    return v;
}

namespace {
// A writer call in progress (batcher_free waits until none is left); ok is false when the batcher
// is closing or gone (the caller must not touch w->b).  The count is taken before `closing` is
// read: either batcher_free sees this call and waits for it, or this call sees `closing`.
struct Inside {
    BwCtl* c;
    bool ok;
    explicit Inside(BwCtl* ctl) : c(ctl) {
        c->inside++;
        ok = !c->closing.load();
    }
    ~Inside() { c->inside--; }
};

int dev_error(BwDev* b) { return set_error(b->error, b->errmsg); }  // errmsg is set before error

BwDev* dev_new(const Algo* a, int device, int index, uint64_t round_bytes, uint32_t max_wait_us) {
    auto* b = new BwDev();
    b->algo = a;
    b->device = device;
    b->index = index;
    b->round_bytes = round_bytes ? round_bytes : (256ull << 20);
    b->writer_cap = std::max<uint64_t>(b->round_bytes / 8, 4ull * kBlock);
    // two arenas per writer, each: the chunk in progress (+ window) and up to four caps of new
    // bytes between compactions (a compaction needs room for the tail and two rounds' bytes)
    b->arena_cap = (a->max_size() + kHist + 4 * (b->writer_cap + kBlock) + 4095) & ~uint64_t(4095);
    b->wait = std::chrono::microseconds(max_wait_us ? max_wait_us : 2000);
    if (a->kind == kFixed) return b;
    Guard g(device);
    int err = 0;
    if (!device_tables(device, &err)) {
        delete b;
        return nullptr;
    }
    // the splits (short, on the round's critical path) go first when both streams have work
    int prio_lo = 0, prio_hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
    hipError_t e = hipStreamCreateWithPriority(&b->stream, hipStreamNonBlocking, prio_hi);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&b->copy, hipStreamNonBlocking);
    for (auto& m : b->meta)
        for (hipEvent_t* ev : {&m.gathered, &m.g0, &m.k0, &m.done})
            if (e == hipSuccess) e = hipEventCreate(ev);
    if (e == hipSuccess) e = hipEventCreate(&b->ev_ref);
    if (e == hipSuccess) e = hipEventRecord(b->ev_ref, b->stream);
    if (e != hipSuccess) {
        hip_err(e, "writer streams");
        delete b;
        return nullptr;
    }
    b->th = std::thread([b] { b->loop(); });
    return b;
}

// Stop the device batcher's round thread (every staged byte is shipped first), then fail every
// later or still-blocked writer call on it.
void dev_stop(BwDev* b) {
    {
        std::lock_guard<std::mutex> lk(b->mu);
        b->stop = true;
    }
    b->cv_round.notify_all();
    if (b->th.joinable()) b->th.join();
    std::lock_guard<std::mutex> lk(b->mu);
    if (!b->error) {
        b->errmsg = "writer batcher closed";
        b->error = KCDC_EINVAL;
    }
    b->cv_done.notify_all();
    for (kcdc_bw* w : b->open) {
        std::lock_guard<std::mutex> wl(w->mu);
        w->cv.notify_all();
    }
}
}  // namespace

extern "C" kcdc_bw_batcher* kcdc_bw_batcher_new_devices(const char* name, const int* devices, int ndev,
                                                        uint64_t round_bytes, uint32_t max_wait_us) {
    const Algo* a = find_algo(name);
    if (!a) {
        set_error(KCDC_ENOENT, std::string("unknown splitter: ") + (name ? name : "(null)"));
        return nullptr;
    }
    std::vector<int> list;
    if (a->kind == kFixed) {  // FIXED reads no data: host arithmetic only, the devices are labels
        if (!devices || ndev <= 0) list.assign(1, 0);
        for (int i = 0; devices && i < ndev; i++) {
            if (devices[i] < 0) {
                set_error(KCDC_ENODEV, "no such HIP device");
                return nullptr;
            }
            list.push_back(devices[i]);
        }
    } else {
        int count = 0;
        if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
            set_error(KCDC_ENODEV, "no HIP device");
            return nullptr;
        }
        if (!devices || ndev <= 0) {
            for (int d = 0; d < count; d++) list.push_back(d);
        } else {
            for (int i = 0; i < ndev; i++) {
                if (devices[i] < 0 || devices[i] >= count) {
                    set_error(KCDC_ENODEV, "no such HIP device");
                    return nullptr;
                }
                list.push_back(devices[i]);
            }
        }
    }
    auto* t = new kcdc_bw_batcher();
    t->algo = a;
    for (size_t i = 0; i < list.size(); i++) {
        BwDev* b = dev_new(a, list[i], static_cast<int>(i), round_bytes, max_wait_us);
        if (!b) {
            for (BwDev* d : t->devs) {
                dev_stop(d);
                delete d;
            }
            delete t;
            return nullptr;
        }
        t->devs.push_back(b);
    }
    return t;
}

extern "C" kcdc_bw_batcher* kcdc_bw_batcher_new(const char* name, int device, uint64_t round_bytes,
                                                uint32_t max_wait_us) {
    return kcdc_bw_batcher_new_devices(name, &device, 1, round_bytes, max_wait_us);
}

extern "C" int kcdc_bw_batcher_devices(const kcdc_bw_batcher* t) {
    return t ? static_cast<int>(t->devs.size()) : set_error(KCDC_EINVAL, "null batcher");
}

extern "C" void kcdc_bw_batcher_free(kcdc_bw_batcher* t) {
    if (!t) return;
    t->ctl->closing = true;
    for (BwDev* b : t->devs) dev_stop(b);
    while (t->ctl->inside.load() > 0) std::this_thread::sleep_for(std::chrono::microseconds(50));
    for (BwDev* b : t->devs) {
        {
            std::lock_guard<std::mutex> lk(b->mu);
            for (kcdc_bw* w : b->open) w->b = nullptr;  // writers not freed: kcdc_bw_free frees their arenas
        }
        if (b->algo->kind != kFixed) {
            Guard g(b->device);
            (void)hipStreamSynchronize(b->stream);
            (void)hipStreamSynchronize(b->copy);
        }
        delete b;
    }
    t->ctl->detached = true;
    delete t;
}

extern "C" kcdc_bw* kcdc_bw_open_hint(kcdc_bw_batcher* t, uint64_t size_hint) {
    if (!t) {
        set_error(KCDC_EINVAL, "null batcher");
        return nullptr;
    }
    Inside in(t->ctl.get());
    if (!in.ok) {
        set_error(KCDC_EINVAL, "writer batcher closed");
        return nullptr;
    }
    // Assign the writer to the device with the least load (bytes of its open writers, each
    // counted as max(size hint, bytes written)): the longest-processing-time rule as bytes
    // arrive (snapshot/upload/upload.go:769-782 runs NumCPU writers against one repository).
    BwDev* b = nullptr;
    {
        std::lock_guard<std::mutex> lk(t->mu);
        for (BwDev* d : t->devs)
            if (!b || d->load.load() < b->load.load()) b = d;
        b->load += size_hint;
    }
    auto* w = new kcdc_bw();
    w->b = b;
    w->ctl = t->ctl;
    w->device = b->device;
    w->hint = size_hint;
    w->counted = size_hint;
    w->fixed_next = b->algo->kind == kFixed ? b->algo->avg : 0;
    if (b->algo->kind != kFixed) {
        Guard g(b->device);
        void *p = nullptr, *q = nullptr;
        {
            std::lock_guard<std::mutex> lk(b->mu);
            if (!b->arenas.empty()) {
                p = b->arenas.back().first;
                q = b->arenas.back().second;
                b->arenas.pop_back();
            }
        }
        hipError_t e = hipSuccess;
        if (!p) e = hipMalloc(&p, b->arena_cap);
        if (e == hipSuccess && !q) e = hipMalloc(&q, b->arena_cap);
        if (e != hipSuccess) {  // give back the cached pairs (another device user may need the memory), retry once
            (void)hipGetLastError();  // (the failed allocation's error is not this call's result)
            {
                std::lock_guard<std::mutex> lk(b->mu);
                b->trim_arenas();
            }
            e = hipSuccess;
            if (!p) e = hipMalloc(&p, b->arena_cap);
            if (e == hipSuccess && !q) e = hipMalloc(&q, b->arena_cap);
        }
        if (e != hipSuccess) {
            if (p) (void)hipFree(p);
            b->load -= size_hint;
            set_error(KCDC_ENOMEM, "writer arenas: 2 x " + std::to_string(b->arena_cap >> 20) +
                                       " MiB of device memory per open writer (" + hipGetErrorString(e) + ")");
            delete w;
            return nullptr;
        }
        w->arena = static_cast<uint8_t*>(p);
        w->spare = static_cast<uint8_t*>(q);
    }
    std::lock_guard<std::mutex> lk(b->mu);
    b->open.push_back(w);
    b->peak_open = std::max(b->peak_open, b->open.size());
    return w;
}

extern "C" kcdc_bw* kcdc_bw_open(kcdc_bw_batcher* t) { return kcdc_bw_open_hint(t, 0); }

extern "C" int kcdc_bw_device(const kcdc_bw* w) {
    return w && w->b ? w->b->index : set_error(KCDC_EINVAL, "writer not open");
}

extern "C" int kcdc_bw_write(kcdc_bw* w, const uint8_t* p, size_t len) {
    if (!w) return set_error(KCDC_EINVAL, "writer not open");
    Inside in(w->ctl.get());
    if (!in.ok) return set_error(KCDC_EINVAL, "writer batcher closed");
    if (!w->b) return set_error(KCDC_EINVAL, "writer not open");
    BwDev* b = w->b;
    if (b->algo->kind == kFixed) {  // splitter_fixed.go:15-26: no data is read
        std::lock_guard<std::mutex> lk(b->mu);
        if (w->finishing) return set_error(KCDC_EINVAL, "write after finish");
        w->written += len;
        if (w->written > w->counted) {
            b->load += w->written - w->counted;
            w->counted = w->written;
        }
        while (w->fixed_next <= w->written) {
            w->ready.push_back(w->fixed_next);
            w->ready_pushed.fetch_add(1, std::memory_order_release);
            w->fixed_next += b->algo->avg;
        }
        return KCDC_OK;
    }
    std::unique_lock<std::mutex> wl(w->mu);
    if (w->finishing) return set_error(KCDC_EINVAL, "write after finish");
    while (len) {
        if (b->error) return dev_error(b);
        // backpressure: at most writer_cap unshipped bytes (a capped writer asks for a round at
        // once: with few writers `staged` may never reach round_bytes)
        if (w->written - w->shipped >= b->writer_cap) {
            const int64_t c0 = now_ns();
            b->capped++;
            b->cv_round.notify_one();
            w->cv.wait(wl, [&] { return b->error || w->written - w->shipped < b->writer_cap; });
            b->capped--;
            b->w_capped_ns += now_ns() - c0;
            continue;
        }
        if (w->blocks.empty() || w->blocks.back().end == kBlock) {
            wl.unlock();  // lock order: the batcher's mutex is never taken under a writer's
            const int64_t g0 = now_ns();
            uint8_t* blk = b->get_block();
            b->w_block_ns += now_ns() - g0;
            wl.lock();
            if (!blk) return set_error(KCDC_ENOMEM, "pinned staging block");
            Blk nb;
            nb.p = blk;
            nb.start = nb.end = static_cast<uint32_t>(w->written & 15u);  // congruent with the arena mod 16
            nb.pos = w->written;
            w->blocks.push_back(nb);
        }
        // Copy without the writer's mutex: a writer preempted inside a 64 KiB copy (more writer
        // threads than CPUs) would hold up the round thread's collection, and with it every writer
        // waiting on the batcher.  Only this thread appends blocks or moves `end`; the round thread
        // never retires the last block while it is partial, so the block stays the last one.
        const size_t k = std::min<size_t>(len, kBlock - w->blocks.back().end);
        uint8_t* dst = w->blocks.back().p + w->blocks.back().end;
        wl.unlock();
        stage_copy(dst, p, k);
        wl.lock();
        Blk& bk = w->blocks.back();
        bk.end += static_cast<uint32_t>(k);
        w->written += k;
        if (w->written > w->counted) {  // bytes beyond the size hint count toward the device's load
            b->load += w->written - w->counted;
            w->counted = w->written;
        }
        const uint64_t before = b->staged.fetch_add(k);
        if (before == 0) b->since = now_ns();
        if (before == 0 || before + k >= b->round_bytes) b->cv_round.notify_one();
        p += k;
        len -= k;
    }
    return KCDC_OK;
}

extern "C" int64_t kcdc_bw_cuts(kcdc_bw* w, uint64_t* out, uint64_t cap) {
    if (!w) return set_error(KCDC_EINVAL, "writer not open");
    Inside in(w->ctl.get());
    if (!in.ok) return set_error(KCDC_EINVAL, "writer batcher closed");
    if (!w->b) return set_error(KCDC_EINVAL, "writer not open");
    BwDev* b = w->b;
    if (b->ids.on) return set_error(KCDC_EINVAL, "content IDs are on: take cuts with kcdc_bw_cuts_ids");
    if (w->ready_pushed.load(std::memory_order_acquire) == w->ready_taken.load(std::memory_order_relaxed) &&
        !b->error)
        return 0;
    std::lock_guard<std::mutex> lk(b->mu);
    const uint64_t avail = w->ready.size() - w->ready_head;
    const uint64_t k = std::min<uint64_t>(avail, cap);
    if (k) std::memcpy(out, w->ready.data() + w->ready_head, k * 8);
    w->ready_head += k;
    w->ready_taken.fetch_add(k, std::memory_order_relaxed);
    if (w->ready_head == w->ready.size()) {
        w->ready.clear();
        w->ready_head = 0;
    }
    if (b->error && k == 0) return dev_error(b);
    return static_cast<int64_t>(k);
}

extern "C" int kcdc_bw_finish(kcdc_bw* w) {
    if (!w) return set_error(KCDC_EINVAL, "writer not open");
    Inside in(w->ctl.get());
    if (!in.ok) return set_error(KCDC_EINVAL, "writer batcher closed");
    if (!w->b) return set_error(KCDC_EINVAL, "writer not open");
    BwDev* b = w->b;
    if (b->algo->kind == kFixed) {
        std::lock_guard<std::mutex> lk(b->mu);
        if (w->finishing) return KCDC_OK;
        const uint64_t last = w->ready.empty() ? w->fixed_next - b->algo->avg : w->ready.back();
        if (w->written > last) {  // the trailing chunk
            w->ready.push_back(w->written);
            w->ready_pushed.fetch_add(1, std::memory_order_release);
        }
        w->finishing = w->done = true;
        return KCDC_OK;
    }
    {
        std::lock_guard<std::mutex> wl(w->mu);
        if (!w->finishing) {
            w->finishing = true;
            b->finish_pending++;
        }
    }
    {
        std::lock_guard<std::mutex> lk(b->mu);  // no lost wakeup: the round thread checks under this mutex
        b->cv_round.notify_one();
    }
    std::unique_lock<std::mutex> lk(b->mu);
    // with content IDs, Result() also waits for the last chunk's name
    b->cv_done.wait(lk, [&] { return (w->done && w->ids_ready == w->ids_made) || b->error; });
    return b->error && !(w->done && w->ids_ready == w->ids_made) ? dev_error(b) : KCDC_OK;
}

extern "C" int64_t kcdc_bw_cuts_ids(kcdc_bw* w, uint64_t* cuts, uint8_t* ids, uint32_t id_stride, uint64_t cap) {
    if (!w) return set_error(KCDC_EINVAL, "writer not open");
    Inside in(w->ctl.get());
    if (!in.ok) return set_error(KCDC_EINVAL, "writer batcher closed");
    if (!w->b) return set_error(KCDC_EINVAL, "writer not open");
    BwDev* b = w->b;
    if (!b->ids.on) return set_error(KCDC_EINVAL, "content IDs are off (kcdc_bw_batcher_hash)");
    if (id_stride < b->ids.out || (cap && (!cuts || !ids))) return set_error(KCDC_EINVAL, "bad ID buffer");
    if (w->ids_pub.load(std::memory_order_acquire) == w->ids_taken.load(std::memory_order_relaxed) && !b->error)
        return 0;
    std::lock_guard<std::mutex> lk(b->mu);
    uint64_t k = 0;
    while (k < cap && !w->ids.empty() && w->ids.front().ready) {
        const kcdc_bw::IdEntry& en = w->ids.front();
        cuts[k] = en.cut;
        std::memcpy(ids + k * id_stride, en.id, b->ids.out);
        w->ids.pop_front();
        w->ids_base++;
        k++;
    }
    w->ids_taken.fetch_add(k, std::memory_order_relaxed);
    if (b->error && k == 0) return dev_error(b);
    return static_cast<int64_t>(k);
}

extern "C" int kcdc_bw_batcher_hash(kcdc_bw_batcher* t, const char* hash_name, const uint8_t* key, uint32_t key_len) {
    if (!t) return set_error(KCDC_EINVAL, "null batcher");
    if (t->algo->kind == kFixed) return set_error(KCDC_EINVAL, "content IDs: FIXED writers stage no bytes on the device");
    std::lock_guard<std::mutex> lk(t->mu);
    for (BwDev* b : t->devs) {
        std::lock_guard<std::mutex> dl(b->mu);
        if (!b->open.empty() || b->rounds) return set_error(KCDC_EINVAL, "content IDs: enable before the first writer opens");
        if (b->ids.on) return set_error(KCDC_EINVAL, "content IDs are already on");
    }
    for (size_t i = 0; i < t->devs.size(); i++) {
        const int rc = t->devs[i]->ids_enable(hash_name, key, key_len);
        if (rc != KCDC_OK) {  // all or nothing: the devices enabled so far go back to plain cuts
            const std::string msg = kcdc_last_error();
            for (size_t k = 0; k <= i; k++) t->devs[k]->ids_disable();
            return set_error(rc, msg);
        }
    }
    return KCDC_OK;
}

extern "C" void kcdc_bw_free(kcdc_bw* w) {
    if (!w) return;
    const std::shared_ptr<BwCtl> ctl = w->ctl;  // (outlives `in`: w and the batcher may hold the last references)
    Inside in(ctl.get());
    if (!in.ok) {  // the batcher is closing: once it has detached this writer, free what is left
        while (!ctl->detached.load()) std::this_thread::sleep_for(std::chrono::microseconds(50));
        if (w->arena) {
            Guard g(w->device);
            (void)hipFree(w->arena);
            (void)hipFree(w->spare);
        }
        delete w;
        return;
    }
    BwDev* b = w->b;
    if (b) {
        // an abandoned object: split (and drop) what it staged, so no round still reads its arena
        if (b->algo->kind != kFixed && !b->error) (void)kcdc_bw_finish(w);
        std::unique_lock<std::mutex> lk(b->mu);
        // a writer whose last round did not complete (an error) may still be in a round the round
        // thread is issuing, or in id_create: wait until it holds no writer pointers
        if (!w->done) b->cv_done.wait(lk, [&] { return b->writer_refs == 0; });
        for (BwDev::Chain& c : b->chains)  // (an error left chains of this writer unnamed)
            if (c.w == w) c.w = nullptr;
        b->load -= std::min<uint64_t>(b->load.load(), w->counted);
        {
            std::lock_guard<std::mutex> pl(b->pool_mu);
            for (Blk& bk : w->blocks) b->pool.push_back(bk.p);
        }
        b->open.erase(std::find(b->open.begin(), b->open.end(), w));
        if (w->arena && w->done && !b->error && b->arenas.size() < b->keep_arenas()) {
            // its last round has completed (finish waited for it), so no gather, compaction or
            // split still touches these arenas
            b->arenas.emplace_back(w->arena, w->spare);
        } else if (w->arena) {
            Guard g(b->device);
            (void)hipStreamSynchronize(b->copy);
            (void)hipStreamSynchronize(b->stream);
            if (b->idcopy) (void)hipStreamSynchronize(b->idcopy);  // (after an error: ring copies may read it)
            (void)hipFree(w->arena);
            (void)hipFree(w->spare);
        }
    } else if (w->arena) {  // its batcher was freed first
        Guard g(w->device);
        (void)hipFree(w->arena);
        (void)hipFree(w->spare);
    }
    delete w;
}

extern "C" int64_t kcdc_bw_rounds(const kcdc_bw_batcher* t) {
    if (!t) return 0;
    int64_t r = 0;
    for (const BwDev* b : t->devs) r += static_cast<int64_t>(b->rounds);
    return r;
}

extern "C" int kcdc_bw_stats(kcdc_bw_batcher* t, double* out, int n) {
    if (!t || !out) return set_error(KCDC_EINVAL, "null argument");
    // per device: the device span from its first round's start to its last one's end, and the
    // part of it in which a gather or a split ran (their union: overlapped rounds count once);
    // over devices: counts and host seconds add up, spans and busy times are the maximum
    double v[24] = {0};
    for (BwDev* b : t->devs) {
        std::lock_guard<std::mutex> lk(b->mu);
        std::vector<std::pair<float, float>> iv = b->busy;
        std::sort(iv.begin(), iv.end());
        double span = 0, busy = 0;
        if (!iv.empty()) {
            float s0 = iv[0].first, e0 = iv[0].second, hi = iv[0].second;
            for (size_t i = 1; i < iv.size(); i++) {
                if (iv[i].first > e0) {
                    busy += e0 - s0;
                    s0 = iv[i].first;
                    e0 = iv[i].second;
                } else {
                    e0 = std::max(e0, iv[i].second);
                }
                hi = std::max(hi, iv[i].second);
            }
            busy += e0 - s0;
            span = hi - iv[0].first;
        }
        const double d[24] = {static_cast<double>(b->rounds), static_cast<double>(b->shipped_bytes), b->t_submit,
                              b->t_wait, b->t_gather, b->t_kernel, span * 1e-3, busy * 1e-3,
                              b->t_seg[0], b->t_seg[1], b->t_seg[2], b->t_seg[3], b->t_seg[4],
                              b->t_idle, b->w_capped_ns.load() * 1e-9, b->w_block_ns.load() * 1e-9,
                              static_cast<double>(b->pool_misses.load()), b->t_lock,
                              static_cast<double>(b->id_chains), static_cast<double>(b->id_steps), b->t_hash,
                              b->t_space, b->t_hidle, static_cast<double>(b->chain_steps)};
        for (int i = 0; i < 24; i++) v[i] = (i == 6 || i == 7) ? std::max(v[i], d[i]) : v[i] + d[i];
    }
    for (int i = 0; i < n && i < 24; i++) out[i] = v[i];
    return 24;
}
