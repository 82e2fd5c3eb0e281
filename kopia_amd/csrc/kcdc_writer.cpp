// Batching object writers (the writer-level remainder): many concurrent
// objectWriter.Write streams (repo/object/object_writer.go:113-139) fed in 64 KiB slices
// (snapshot/upload/upload.go:394-407) are accumulated per writer in pinned host staging and
// split together: one round = every writer's new bytes up in one burst of H2D copies, one
// batch-splitter launch over all writers' unresolved regions, their cut lists back.  Each
// byte crosses PCIe once; a writer's unresolved tail (the chunk in progress plus the 64-byte
// window before it) stays on the device from round to round.
//
// Exactness: the rolling hash at position p is a function of the 64 bytes ending at p
// (SURVEY.md §0.4), and a chunk's cut is the first candidate in [s+min-1, s+max-1] (or the
// forced cut).  A round splits region [tail_pos, shipped) starting its first chunk at the
// writer's last final cut (kernel `starts`: the bytes before it are window history only).
// Every cut it reports is final except the last one, which is the region end (the chunk
// still growing), unless the writer is finishing.  So the cuts equal one NextSplitPoint pass
// over the whole object, however the bytes were sliced (tests/test_gpu_writer.py).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/kcdc.h"
#include "kcdc_internal.h"

using namespace kcdc;

namespace {

constexpr size_t kBlock = 4u << 20;  // pinned staging block (one H2D copy each)
constexpr uint64_t kHist = 64;       // window history kept before a writer's last final cut

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

uint64_t align16(uint64_t x) { return (x + 15) & ~uint64_t(15); }

}  // namespace

struct kcdc_bw;

struct kcdc_bw_batcher {
    const Algo* algo = nullptr;
    int device = 0;
    uint64_t round_bytes = 0;    // ship once this many new bytes are staged across writers
    uint64_t writer_cap = 0;     // a writer blocks in write() while this many of its bytes are unshipped
    std::chrono::microseconds wait{0};
    hipStream_t stream = nullptr;

    std::mutex mu;
    std::condition_variable cv_round;  // round thread: work arrived
    std::condition_variable cv_done;   // writers: a round finished
    std::vector<kcdc_bw*> open;        // writers not yet freed
    std::vector<uint8_t*> pool;        // free pinned blocks
    uint64_t staged = 0;               // unshipped bytes over all writers
    std::chrono::steady_clock::time_point since;  // when `staged` last became nonzero
    uint32_t capped = 0;               // writers blocked on their staging cap (a round is due)
    uint64_t rounds = 0;
    // observability (kcdc_bw_stats): bytes shipped, seconds in the round thread's phases
    uint64_t shipped_bytes = 0;
    double t_submit = 0, t_wait = 0;
    bool stop = false;
    int error = 0;
    std::string errmsg;
    std::thread th;

    // device: ping-pong region buffers (tails + new bytes of every writer), metadata
    uint8_t* dreg[2] = {nullptr, nullptr};
    size_t dreg_cap[2] = {0, 0};
    int cur = 0;
    uint64_t* dmeta = nullptr;  // ptrs | lens | starts | cut_base | counts | cuts
    size_t dmeta_cap = 0;
    uint64_t* hmeta = nullptr;  // pinned mirror
    size_t hmeta_cap = 0;

    ~kcdc_bw_batcher() {
        Guard g(device);
        for (uint8_t* b : pool) (void)hipHostFree(b);
        for (auto* p : dreg)
            if (p) (void)hipFree(p);
        if (dmeta) (void)hipFree(dmeta);
        if (hmeta) (void)hipHostFree(hmeta);
        if (stream) (void)hipStreamDestroy(stream);
    }
    uint8_t* get_block() {  // mu held
        if (!pool.empty()) {
            uint8_t* b = pool.back();
            pool.pop_back();
            return b;
        }
        void* p = nullptr;
        Guard g(device);
        return hipHostMalloc(&p, kBlock, hipHostMallocDefault) == hipSuccess ? static_cast<uint8_t*>(p) : nullptr;
    }
    int run_round(std::unique_lock<std::mutex>& lk);
    void loop();
};

struct kcdc_bw {
    kcdc_bw_batcher* b = nullptr;
    // host staging: bytes [shipped, written) in blocks (the last one filled up to `fill`)
    std::vector<uint8_t*> blocks;
    size_t fill = 0;
    uint64_t written = 0, shipped = 0;
    // device tail: stream bytes [tail_pos, shipped) at dtail (inside the batcher's region buffer)
    const uint8_t* dtail = nullptr;
    uint64_t tail_pos = 0;
    uint64_t frontier = 0;          // last final cut (0: none yet)
    std::vector<uint64_t> ready;    // final cuts not taken yet
    size_t ready_head = 0;
    bool finishing = false, done = false;
    bool copying = false;           // write() is copying into its last block (lock dropped)
    uint64_t fixed_next = 0;        // FIXED names: the next cut (no data is read)
};

// One round (called by the round thread with `lk` held; drops it while the device works).
int kcdc_bw_batcher::run_round(std::unique_lock<std::mutex>& lk) {
    struct Job {
        kcdc_bw* w;
        std::vector<uint8_t*> blocks;
        uint64_t new_bytes, tail_len, off;  // off: region offset in the new buffer
        bool finishing, launch;
    };
    std::vector<Job> jobs;
    for (kcdc_bw* w : open) {
        if (w->done) continue;
        if (w->copying) {  // its staged bytes wait for the next round; the tail still moves
            if (w->shipped > w->tail_pos) jobs.push_back(Job{w, {}, 0, w->shipped - w->tail_pos, 0, false, false});
            continue;
        }
        Job j{w, {}, w->written - w->shipped, w->shipped - w->tail_pos, 0, w->finishing, false};
        j.blocks.swap(w->blocks);
        w->fill = 0;
        w->shipped = w->written;
        staged -= j.new_bytes;
        // launch it when it has new bytes past what a final cut could need, or finishes
        j.launch = j.finishing || j.new_bytes > 0;
        if (j.launch || j.tail_len) jobs.push_back(std::move(j));
    }
    rounds++;
    lk.unlock();
    cv_done.notify_all();  // writers blocked on their staging cap may continue

    int rc = KCDC_OK;
    uint64_t total = 0, fresh = 0;
    for (Job& j : jobs) {
        j.off = total;
        total += align16(j.tail_len + j.new_bytes);
        fresh += j.new_bytes;
    }
    const auto t0 = std::chrono::steady_clock::now();
    const int nxt = cur ^ 1;
    Guard g(device);
    auto fail = [&](hipError_t e, const char* what) { rc = hip_err(e, what); };
    if (dreg_cap[nxt] < total) {
        if (dreg[nxt]) (void)hipFree(dreg[nxt]);
        dreg[nxt] = nullptr;
        dreg_cap[nxt] = 0;
        const size_t want = std::max<size_t>(total + total / 4, 64u << 20);
        hipError_t e = hipMalloc(&dreg[nxt], want);
        if (e != hipSuccess) fail(e, "writer region buffer");
        else dreg_cap[nxt] = want;
    }
    std::vector<uint32_t> li;  // jobs launched
    for (uint32_t i = 0; i < jobs.size(); i++)
        if (jobs[i].launch) li.push_back(i);
    const uint32_t n = static_cast<uint32_t>(li.size());
    uint64_t cuts_cap = 0;
    std::vector<uint64_t> cbase(n);
    for (uint32_t k = 0; k < n; k++) {
        const Job& j = jobs[li[k]];
        cbase[k] = cuts_cap;
        cuts_cap += (j.tail_len + j.new_bytes) / algo->min_size() + 2;
    }
    const size_t meta_words = 5ull * n + cuts_cap + 1;
    if (rc == KCDC_OK && dmeta_cap < meta_words) {
        if (dmeta) (void)hipFree(dmeta);
        if (hmeta) (void)hipHostFree(hmeta);
        dmeta = hmeta = nullptr;
        dmeta_cap = hmeta_cap = 0;
        const size_t want = std::max<size_t>(meta_words * 2, 1u << 16);
        hipError_t e = hipMalloc(&dmeta, want * 8);
        if (e == hipSuccess) e = hipHostMalloc(&hmeta, want * 8, hipHostMallocDefault);
        if (e != hipSuccess) fail(e, "writer metadata");
        else dmeta_cap = hmeta_cap = want;
    }
    if (rc == KCDC_OK) {
        // tails (device to device) and new bytes (pinned host to device) into the new buffer
        for (Job& j : jobs) {
            uint8_t* dst = dreg[nxt] + j.off;
            if (j.tail_len && rc == KCDC_OK) {
                hipError_t e = hipMemcpyAsync(dst, j.w->dtail, j.tail_len, hipMemcpyDeviceToDevice, stream);
                if (e != hipSuccess) fail(e, "writer tail copy");
            }
            uint64_t left = j.new_bytes, at = j.tail_len;
            for (uint8_t* blk : j.blocks) {
                const size_t k = left < kBlock ? static_cast<size_t>(left) : kBlock;
                if (k && rc == KCDC_OK) {
                    hipError_t e = hipMemcpyAsync(dst + at, blk, k, hipMemcpyHostToDevice, stream);
                    if (e != hipSuccess) fail(e, "writer H2D");
                }
                at += k;
                left -= k;
            }
        }
    }
    uint64_t* hp = hmeta;
    if (rc == KCDC_OK && n) {
        uint64_t* dp = dmeta;
        for (uint32_t k = 0; k < n; k++) {
            const Job& j = jobs[li[k]];
            hp[k] = reinterpret_cast<uint64_t>(dreg[nxt] + j.off);                 // ptrs
            hp[n + k] = j.tail_len + j.new_bytes;                                  // lens
            hp[2 * n + k] = j.w->frontier - j.w->tail_pos;                         // starts
            hp[3 * n + k] = cbase[k];                                              // cut_base
        }
        hipError_t e = hipMemcpyAsync(dp, hp, 4ull * n * 8, hipMemcpyHostToDevice, stream);
        if (e != hipSuccess) fail(e, "writer metadata H2D");
        if (rc == KCDC_OK) {
            SplitArgs s;
            s.ptrs = reinterpret_cast<const uint8_t* const*>(dp);
            s.lens = dp + n;
            s.starts = dp + 2 * n;
            s.cut_base = dp + 3 * n;
            s.counts = dp + 4 * n;
            s.cuts = dp + 5 * n;
            s.cuts_cap = cuts_cap;
            s.nstreams = n;
            rc = launch_split_batch(*algo, s, device, stream);
        }
        if (rc == KCDC_OK) {
            e = hipMemcpyAsync(hp + 4 * n, dp + 4 * n, (n + cuts_cap) * 8, hipMemcpyDeviceToHost, stream);
            if (e != hipSuccess) fail(e, "writer cuts D2H");
        }
    }
    const auto t1 = std::chrono::steady_clock::now();
    if (rc == KCDC_OK) {
        hipError_t e = hipStreamSynchronize(stream);
        if (e != hipSuccess) fail(e, "writer round");
    }
    const auto t2 = std::chrono::steady_clock::now();

    lk.lock();
    shipped_bytes += fresh;
    t_submit += std::chrono::duration<double>(t1 - t0).count();
    t_wait += std::chrono::duration<double>(t2 - t1).count();
    for (Job& j : jobs)  // the H2D copies have completed (or failed): blocks back to the pool
        for (uint8_t* blk : j.blocks) pool.push_back(blk);
    if (rc != KCDC_OK) return rc;
    for (uint32_t k = 0; k < n; k++) {
        Job& j = jobs[li[k]];
        kcdc_bw* w = j.w;
        const uint64_t cnt = hp[4 * n + k];
        if (cnt == ~0ull || cnt > (j.tail_len + j.new_bytes) / algo->min_size() + 2)
            return set_error(KCDC_EIO, "writer round: the device lost a stream");
        const uint64_t* c = hp + 5 * n + cbase[k];
        const uint64_t fin = j.finishing ? cnt : (cnt ? cnt - 1 : 0);
        for (uint64_t t = 0; t < fin; t++) w->ready.push_back(w->tail_pos + c[t]);
        if (fin) w->frontier = w->tail_pos + c[fin - 1];
        if (j.finishing) w->done = true;
    }
    for (Job& j : jobs) {  // new tails: [frontier - 64, shipped) inside the new buffer
        kcdc_bw* w = j.w;
        const uint64_t keep = w->frontier >= kHist ? w->frontier - kHist : 0;
        w->dtail = dreg[nxt] + j.off + (keep - w->tail_pos);
        w->tail_pos = keep;
    }
    cur = nxt;
    return KCDC_OK;
}

void kcdc_bw_batcher::loop() {
    std::unique_lock<std::mutex> lk(mu);
    auto last = std::chrono::steady_clock::now();
    for (;;) {
        auto work = [&] {
            if (stop || error) return true;
            if (staged >= round_bytes || capped) return true;
            for (kcdc_bw* w : open)
                if (w->finishing && !w->done) return true;
            return false;
        };
        // Ship when a round's worth is staged, a writer is blocked on its cap or finishing, or
        // max_wait after the first unshipped byte (or after the last round) -- whichever is first.
        // Writers wake this thread when `staged` leaves 0, so the timed wait always starts.
        while (!work()) {
            if (staged > 0) {
                const auto due = std::max(last, since) + wait;
                if (cv_round.wait_until(lk, due, work)) break;
                if (std::chrono::steady_clock::now() >= due) break;
            } else {
                cv_round.wait(lk, [&] { return work() || staged > 0; });
            }
        }
        if (stop && staged == 0) {
            bool pending = false;
            for (kcdc_bw* w : open) pending = pending || (w->finishing && !w->done);
            if (!pending) break;
        }
        if (error) break;
        if (staged == 0) {
            bool pending = false;
            for (kcdc_bw* w : open) pending = pending || (w->finishing && !w->done);
            if (!pending) continue;
        }
        const int rc = run_round(lk);
        last = std::chrono::steady_clock::now();
        if (rc != KCDC_OK) {
            error = rc;
            errmsg = kcdc_last_error();
        }
        cv_done.notify_all();
    }
    cv_done.notify_all();
}

extern "C" kcdc_bw_batcher* kcdc_bw_batcher_new(const char* name, int device, uint64_t round_bytes,
                                                uint32_t max_wait_us) {
    const Algo* a = find_algo(name);
    if (!a) {
        set_error(KCDC_ENOENT, std::string("unknown splitter: ") + (name ? name : "(null)"));
        return nullptr;
    }
    int n = 0;
    if (a->kind != kFixed && (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n)) {
        set_error(KCDC_ENODEV, "no such HIP device");  // FIXED reads no data: host arithmetic only
        return nullptr;
    }
    auto* b = new kcdc_bw_batcher();
    b->algo = a;
    b->device = device;
    b->round_bytes = round_bytes ? round_bytes : (256ull << 20);
    b->writer_cap = std::max<uint64_t>(b->round_bytes / 2, 4ull * kBlock);
    b->wait = std::chrono::microseconds(max_wait_us ? max_wait_us : 2000);
    if (a->kind != kFixed) {
        Guard g(device);
        int err = 0;
        if (!device_tables(device, &err)) {
            delete b;
            return nullptr;
        }
        hipError_t e = hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking);
        if (e != hipSuccess) {
            hip_err(e, "writer stream");
            delete b;
            return nullptr;
        }
        b->th = std::thread([b] { b->loop(); });
    }
    return b;
}

extern "C" void kcdc_bw_batcher_free(kcdc_bw_batcher* b) {
    if (!b) return;
    {
        std::lock_guard<std::mutex> lk(b->mu);
        b->stop = true;
    }
    b->cv_round.notify_all();
    if (b->th.joinable()) b->th.join();
    for (kcdc_bw* w : b->open) w->b = nullptr;  // writers not freed: unusable from now on
    delete b;
}

extern "C" kcdc_bw* kcdc_bw_open(kcdc_bw_batcher* b) {
    if (!b) {
        set_error(KCDC_EINVAL, "null batcher");
        return nullptr;
    }
    auto* w = new kcdc_bw();
    w->b = b;
    w->fixed_next = b->algo->kind == kFixed ? b->algo->avg : 0;
    std::lock_guard<std::mutex> lk(b->mu);
    b->open.push_back(w);
    return w;
}

extern "C" int kcdc_bw_write(kcdc_bw* w, const uint8_t* p, size_t len) {
    if (!w || !w->b) return set_error(KCDC_EINVAL, "writer not open");
    kcdc_bw_batcher* b = w->b;
    std::unique_lock<std::mutex> lk(b->mu);
    if (w->finishing) return set_error(KCDC_EINVAL, "write after finish");
    if (b->error) return set_error(b->error, b->errmsg);
    if (b->algo->kind == kFixed) {  // splitter_fixed.go:15-26: no data is read
        w->written += len;
        while (w->fixed_next <= w->written) {
            w->ready.push_back(w->fixed_next);
            w->fixed_next += b->algo->avg;
        }
        return KCDC_OK;
    }
    while (len) {
        // backpressure: at most writer_cap unshipped bytes per writer (a capped writer asks for
        // a round at once: with few writers `staged` may never reach round_bytes)
        if (w->written - w->shipped >= b->writer_cap) {
            b->capped++;
            b->cv_round.notify_one();
            b->cv_done.wait(lk, [&] { return b->error || w->written - w->shipped < b->writer_cap; });
            b->capped--;
        }
        if (b->error) return set_error(b->error, b->errmsg);
        if (w->blocks.empty() || w->fill == kBlock) {
            uint8_t* blk = b->get_block();
            if (!blk) return set_error(KCDC_ENOMEM, "pinned staging block");
            w->blocks.push_back(blk);
            w->fill = 0;
        }
        const size_t k = std::min(len, kBlock - w->fill);
        uint8_t* dst = w->blocks.back() + w->fill;
        // Copy outside the lock; while `copying` the round thread leaves this writer's blocks
        // alone (it still moves the device tail), and the bytes count only once they landed.
        w->copying = true;
        lk.unlock();
        std::memcpy(dst, p, k);
        lk.lock();
        w->copying = false;
        w->fill += k;
        w->written += k;
        const bool first = b->staged == 0;
        if (first) b->since = std::chrono::steady_clock::now();
        b->staged += k;
        if (first || b->staged >= b->round_bytes) b->cv_round.notify_one();
        p += k;
        len -= k;
    }
    return KCDC_OK;
}

extern "C" int64_t kcdc_bw_cuts(kcdc_bw* w, uint64_t* out, uint64_t cap) {
    if (!w || !w->b) return set_error(KCDC_EINVAL, "writer not open");
    std::lock_guard<std::mutex> lk(w->b->mu);
    const uint64_t avail = w->ready.size() - w->ready_head;
    const uint64_t k = std::min<uint64_t>(avail, cap);
    if (k) std::memcpy(out, w->ready.data() + w->ready_head, k * 8);
    w->ready_head += k;
    if (w->ready_head == w->ready.size()) {
        w->ready.clear();
        w->ready_head = 0;
    }
    if (w->b->error && k == 0) return set_error(w->b->error, w->b->errmsg);
    return static_cast<int64_t>(k);
}

extern "C" int kcdc_bw_finish(kcdc_bw* w) {
    if (!w || !w->b) return set_error(KCDC_EINVAL, "writer not open");
    kcdc_bw_batcher* b = w->b;
    std::unique_lock<std::mutex> lk(b->mu);
    if (b->algo->kind == kFixed) {
        const uint64_t last = w->ready.empty() ? w->fixed_next - b->algo->avg : w->ready.back();
        if (w->written > last) w->ready.push_back(w->written);  // the trailing chunk
        w->finishing = w->done = true;
        return KCDC_OK;
    }
    // A staging copy that raced the lock must have landed: calls on one writer are serialised.
    w->finishing = true;
    b->cv_round.notify_one();
    b->cv_done.wait(lk, [&] { return w->done || b->error; });
    return b->error && !w->done ? set_error(b->error, b->errmsg) : KCDC_OK;
}

extern "C" void kcdc_bw_free(kcdc_bw* w) {
    if (!w) return;
    kcdc_bw_batcher* b = w->b;
    if (b) {
        std::unique_lock<std::mutex> lk(b->mu);
        if (!w->done && b->algo->kind != kFixed && !b->error) {  // abandoned object: drop its bytes
            w->finishing = true;
            b->cv_round.notify_one();
            b->cv_done.wait(lk, [&] { return w->done || b->error; });
        }
        for (uint8_t* blk : w->blocks) b->pool.push_back(blk);
        if (!w->done) b->staged -= w->written - w->shipped;
        b->open.erase(std::find(b->open.begin(), b->open.end(), w));
    }
    delete w;
}

extern "C" int64_t kcdc_bw_rounds(const kcdc_bw_batcher* b) { return b ? static_cast<int64_t>(b->rounds) : 0; }

extern "C" int kcdc_bw_stats(kcdc_bw_batcher* b, double* out, int n) {
    if (!b || !out) return set_error(KCDC_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(b->mu);
    const double v[4] = {static_cast<double>(b->rounds), static_cast<double>(b->shipped_bytes), b->t_submit, b->t_wait};
    for (int i = 0; i < n && i < 4; i++) out[i] = v[i];
    return 4;
}
