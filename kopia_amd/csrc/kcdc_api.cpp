// C ABI of libkcdc (include/kcdc.h): the drop-in boundary for Kopia's
// repo/splitter package.  Host orchestration only; every byte of hashing runs
// in the gfx950 kernels of kcdc_kernels.hip.  There is no CPU fallback.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

#include "../../include/kcdc.h"
#include "kcdc_internal.h"

namespace kcdc {
const char* last_error_cstr();
}

using namespace kcdc;

namespace {

int hip_err(hipError_t e, const char* what) { return set_error(KCDC_EIO, std::string(what) + ": " + hipGetErrorString(e)); }

#define HIP_TRY(expr, what)                          \
    do {                                             \
        hipError_t e_ = (expr);                      \
        if (e_ != hipSuccess) return hip_err(e_, what); \
    } while (0)

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

bool is_gfx950(int dev) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, dev) != hipSuccess) return false;
    return std::strncmp(p.gcnArchName, "gfx950", 6) == 0;
}

int check_device(int dev) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return set_error(KCDC_ENODEV, "no HIP device visible");
    if (dev < 0 || dev >= n) return set_error(KCDC_ENODEV, "device index out of range");
    if (!is_gfx950(dev)) return set_error(KCDC_ENODEV, "device is not gfx950 (MI355X); kernels are gfx950-only");
    return KCDC_OK;
}

}  // namespace

// ======================================================= diagnostics / registry
extern "C" const char* kcdc_last_error(void) { return kcdc::last_error_cstr(); }
extern "C" const char* kcdc_version(void) {
    static const std::string v = [] {
        std::string a = std::string(ablations_kernels()) + ablations_crypt();
        if (!a.empty()) a.pop_back();
        return std::string("kcdc 0.3 (gfx950) ablations=") + (a.empty() ? "none" : a);
    }();
    return v.c_str();
}

extern "C" int kcdc_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    int c = 0;
    for (int i = 0; i < n; i++) c += is_gfx950(i) ? 1 : 0;
    return c;
}

extern "C" int kcdc_supported_algorithms(const char** names, int cap) {
    const int n = algo_count();
    for (int i = 0; names && i < n && i < cap; i++) names[i] = algo_at(i).name;
    return n;
}

extern "C" const char* kcdc_default_algorithm(void) { return "DYNAMIC-4M-BUZHASH"; }

extern "C" int kcdc_lookup(const char* name, kcdc_algo_info* info) {
    const Algo* a = find_algo(name);
    if (!a) return set_error(KCDC_ENOENT, std::string("unknown splitter: ") + (name ? name : "(null)"));
    if (info) {
        info->kind = a->kind;
        info->pooled = a->pooled ? 1 : 0;
        info->avg = a->avg;
        info->min_size = a->min_size();
        info->max_size = a->max_size();
        info->mask = a->mask();
    }
    return KCDC_OK;
}

extern "C" int64_t kcdc_max_segment_size(const char* name) {
    const Algo* a = find_algo(name);
    if (!a) return set_error(KCDC_ENOENT, std::string("unknown splitter: ") + (name ? name : "(null)"));
    return static_cast<int64_t>(a->max_size());
}

extern "C" const char* kcdc_custom_algorithm(int32_t kind, uint64_t avg) {
    const Algo* a = custom_algo(kind, avg);
    if (!a) {
        set_error(KCDC_EINVAL, "invalid custom splitter parameters");
        return nullptr;
    }
    return a->name;
}

extern "C" uint64_t kcdc_cut_capacity(const char* name, uint64_t len) {
    const Algo* a = find_algo(name);
    if (!a) return 0;
    return len / a->min_size() + 1;
}

extern "C" int kcdc_tables(uint32_t* buz, uint64_t* pol, uint64_t* out, uint64_t* mod) {
    const Tables& t = tables();
    if (buz) std::memcpy(buz, t.buz, sizeof(t.buz));
    if (pol) *pol = t.rk_pol;
    if (out) std::memcpy(out, t.rk_out, sizeof(t.rk_out));
    if (mod) std::memcpy(mod, t.rk_mod, sizeof(t.rk_mod));
    return KCDC_OK;
}

// ============================================================ streaming handle
struct kcdc_splitter {
    const Algo* algo = nullptr;
    int device = 0;
    hipStream_t stream = nullptr;
    int64_t count = 0;              // rs.count (rolling) / s.cur (fixed)
    uint8_t hist[kWindow] = {0};    // last 64 stream bytes (zeros before the start)
    uint8_t* h_stage = nullptr;     // pinned: hist || slice
    uint8_t* d_stage = nullptr;
    uint8_t* d_scratch = nullptr;   // zero-copy: device memory the fallback scan copies the staging into
    size_t stage_cap = 0;
    int64_t* d_out = nullptr;
    int64_t* h_out = nullptr;
    kcdc_group* group = nullptr;  // set: GPU scans are batched with the group's other handles
};

#ifndef KCDC_HANDLE_ZC
#define KCDC_HANDLE_ZC 1  // private handles: the scan reads the pinned staging in place (mapped)
#endif

namespace {

struct Pool {
    std::mutex mu;
    std::vector<kcdc_splitter*> free;
};
Pool g_pools[64];

void push_hist(kcdc_splitter* s, const uint8_t* b, size_t n) {
    if (n >= static_cast<size_t>(kWindow)) {
        std::memcpy(s->hist, b + n - kWindow, kWindow);
    } else if (n > 0) {
        std::memmove(s->hist, s->hist + n, kWindow - n);
        std::memcpy(s->hist + kWindow - n, b, n);
    }
}

void destroy(kcdc_splitter* s) {
    if (!s) return;
    DeviceGuard g(s->device);
    if (s->d_stage && !KCDC_HANDLE_ZC) (void)hipFree(s->d_stage);  // zero-copy: a mapping of h_stage
    if (s->h_stage) (void)hipHostFree(s->h_stage);
    if (s->d_scratch) (void)hipFree(s->d_scratch);
    if (s->d_out && !KCDC_HANDLE_ZC) (void)hipFree(s->d_out);
    if (s->h_out) (void)hipHostFree(s->h_out);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    delete s;
}

// The one-word answer of a private scan (zero-copy: written by the kernel into mapped host memory).
hipError_t alloc_out(kcdc_splitter* s) {
    if (KCDC_HANDLE_ZC) {
        hipError_t e = hipHostMalloc(&s->h_out, sizeof(int64_t), hipHostMallocMapped);
        void* pd = nullptr;
        if (e == hipSuccess) e = hipHostGetDevicePointer(&pd, s->h_out, 0);
        s->d_out = static_cast<int64_t*>(pd);
        return e;
    }
    hipError_t e = hipMalloc(&s->d_out, sizeof(int64_t));
    if (e == hipSuccess) e = hipHostMalloc(&s->h_out, sizeof(int64_t), hipHostMallocDefault);
    return e;
}

int ensure_stage(kcdc_splitter* s, size_t need) {
    if (need <= s->stage_cap) return KCDC_OK;
    size_t cap = std::max<size_t>(need, 1 << 20);
    cap = std::min<size_t>(std::max(cap, s->stage_cap * 2), s->algo->max_size() + 2 * kWindow);
    cap = std::max(cap, need);
    if (s->d_stage && !KCDC_HANDLE_ZC) (void)hipFree(s->d_stage);
    if (s->h_stage) (void)hipHostFree(s->h_stage);
    if (s->d_scratch) (void)hipFree(s->d_scratch);
    s->d_stage = nullptr;
    s->h_stage = nullptr;
    s->d_scratch = nullptr;
    s->stage_cap = 0;
    if (KCDC_HANDLE_ZC) {
        // fine-grained: the resident scan server reads it between requests without a kernel
        // boundary, so no stale cached copy may survive
        HIP_TRY(hipHostMalloc(&s->h_stage, cap, hipHostMallocMapped | hipHostMallocCoherent), "hipHostMalloc stage");
        void* pd = nullptr;
        HIP_TRY(hipHostGetDevicePointer(&pd, s->h_stage, 0), "stage mapping");
        s->d_stage = static_cast<uint8_t*>(pd);
        HIP_TRY(hipMalloc(&s->d_scratch, cap), "hipMalloc scan scratch");
    } else {
        HIP_TRY(hipMalloc(&s->d_stage, cap), "hipMalloc stage");
        HIP_TRY(hipHostMalloc(&s->h_stage, cap, hipHostMallocDefault), "hipHostMalloc stage");
    }
    s->stage_cap = cap;
    return KCDC_OK;
}

int64_t group_first_candidate(kcdc_splitter* s, const uint8_t* b, size_t n);
void group_handle_closed(kcdc_group* g);

std::atomic<int> g_open_private{0};  // open private handles of the dynamic splitters (all devices)

// First candidate index in slice b[0..n) given the 64-byte history, on the GPU.
int64_t gpu_first_candidate(kcdc_splitter* s, const uint8_t* b, size_t n) {
    if (s->group) {
        const int64_t f = group_first_candidate(s, b, n);
        if (f != KCDC_EOVERFLOW) return f;  // too big for the group's staging: scan it alone
    }
    const size_t total = kWindow + n;
    int rc = ensure_stage(s, total);
    if (rc) return rc;
    std::memcpy(s->h_stage, s->hist, kWindow);
    std::memcpy(s->h_stage + kWindow, b, n);
    if (KCDC_HANDLE_ZC) {
        // The resident scan server (no launch, tables already in LDS) when this is the only open
        // private handle: the server is one workgroup, so concurrent writers would queue on it,
        // while launches of their own run side by side (16 writers: 12.5 GB/s launching, 7.1
        // through the server).
        if (g_open_private.load(std::memory_order_acquire) == 1) {
            int64_t f = -1;
            const int rs = server_scan_first(*s->algo, s->d_stage, total, kWindow, static_cast<int64_t>(total) - 1,
                                             s->device, &f);
            if (rs < 0) return rs;
            if (rs == 0) return f < 0 ? -1 : f - kWindow;
        }
        // other scans in flight, or the server is busy or unavailable: a launch of our own
    }
    if (!KCDC_HANDLE_ZC)
        HIP_TRY(hipMemcpyAsync(s->d_stage, s->h_stage, total, hipMemcpyHostToDevice, s->stream), "H2D slice");
    rc = launch_scan_first(*s->algo, s->d_stage, total, kWindow, static_cast<int64_t>(total) - 1, s->d_out, s->device,
                           s->stream, s->d_scratch);
    if (rc) return rc;
    if (!KCDC_HANDLE_ZC)
        HIP_TRY(hipMemcpyAsync(s->h_out, s->d_out, sizeof(int64_t), hipMemcpyDeviceToHost, s->stream), "D2H result");
    HIP_TRY(hipStreamSynchronize(s->stream), "scan sync");
    const int64_t f = s->h_out[0];
    return f < 0 ? -1 : f - kWindow;
}

}  // namespace

extern "C" kcdc_splitter* kcdc_splitter_new(const char* name, int device) {
    const Algo* a = find_algo(name);
    if (!a) {
        set_error(KCDC_ENOENT, std::string("unknown splitter: ") + (name ? name : "(null)"));
        return nullptr;
    }
    if (a->kind != kFixed && check_device(device) != KCDC_OK) return nullptr;
    const int idx = algo_index(a);
    if (a->pooled && idx >= 0) {  // pooled(): reuse a Reset splitter (splitter_pool.go:24-30)
        Pool& p = g_pools[idx];
        std::lock_guard<std::mutex> lk(p.mu);
        for (size_t i = 0; i < p.free.size(); i++) {
            if (p.free[i]->device == device) {
                kcdc_splitter* s = p.free[i];
                p.free.erase(p.free.begin() + static_cast<long>(i));
                if (a->kind != kFixed) g_open_private.fetch_add(1, std::memory_order_acq_rel);
                return s;
            }
        }
    }
    kcdc_splitter* s = new kcdc_splitter();
    s->algo = a;
    s->device = device;
    if (a->kind != kFixed) {
        DeviceGuard g(device);
        int err = 0;
        if (!device_tables(device, &err) || hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess ||
            alloc_out(s) != hipSuccess) {
            if (!err) set_error(KCDC_EIO, "failed to allocate splitter device resources");
            destroy(s);
            return nullptr;
        }
        g_open_private.fetch_add(1, std::memory_order_acq_rel);
    }
    return s;
}

extern "C" int64_t kcdc_splitter_next(kcdc_splitter* s, const uint8_t* b, size_t len) {
    if (!s) return set_error(KCDC_EINVAL, "null splitter");
    if (len > 0 && !b) return set_error(KCDC_EINVAL, "null buffer");
    const Algo& A = *s->algo;
    const int64_t n = static_cast<int64_t>(len);
    if (A.kind == kFixed) {  // splitter_fixed.go:15-26 (reads no data)
        const int64_t need = static_cast<int64_t>(A.avg) - s->count;
        if (n < need) {
            s->count += n;
            return -1;
        }
        s->count = 0;
        return need;
    }
    DeviceGuard g(s->device);
    const int64_t mn = static_cast<int64_t>(A.min_size()), mx = static_cast<int64_t>(A.max_size());
    int64_t fast = 0;
    const uint8_t* p = b;
    int64_t rest = n;
    int64_t left = mn - s->count - 1;
    if (left > 0) {  // :29-40 below min size no position is tested; only the window moves
        fast = std::min(left, rest);
        push_hist(s, p, static_cast<size_t>(fast));
        s->count += fast;
        p += fast;
        rest -= fast;
    }
    left = mx - s->count;
    if (left > 0) {  // :42-58 test positions on the GPU
        const int64_t fp = std::min(left, rest);
        if (fp > 0) {
            const int64_t f = gpu_first_candidate(s, p, static_cast<size_t>(fp));
            if (f < -1) return f;  // error code
            if (f >= 0) {
                push_hist(s, p, static_cast<size_t>(f + 1));
                s->count = 0;
                return fast + f + 1;
            }
            push_hist(s, p, static_cast<size_t>(fp));
            s->count += fp;
            fast += fp;
        }
    }
    if (s->count >= mx) {  // :60-64
        s->count = 0;
        return fast;
    }
    return -1;
}

extern "C" int64_t kcdc_splitter_max_segment_size(const kcdc_splitter* s) {
    return s ? static_cast<int64_t>(s->algo->max_size()) : KCDC_EINVAL;
}

extern "C" void kcdc_splitter_reset(kcdc_splitter* s) {
    if (!s) return;
    s->count = 0;
    std::memset(s->hist, 0, sizeof s->hist);
}

extern "C" void kcdc_splitter_close(kcdc_splitter* s) {
    if (!s) return;
    kcdc_splitter_reset(s);  // recyclableSplitter.Close: Reset, then pool.Put
    if (s->group) {  // grouped handles are never pooled
        group_handle_closed(s->group);
        destroy(s);
        return;
    }
    if (s->algo->kind != kFixed) g_open_private.fetch_sub(1, std::memory_order_acq_rel);
    if (s->algo->pooled && algo_index(s->algo) >= 0) {
        Pool& p = g_pools[algo_index(s->algo)];
        std::lock_guard<std::mutex> lk(p.mu);
        p.free.push_back(s);
        return;
    }
    destroy(s);
}

// ============================================== grouped streaming handles
// Many object writers run at once (snapshot/upload/upload.go:769-782), each calling
// NextSplitPoint on its own splitter with a 64 KiB slice.  Alone, each call is one GPU
// round trip.  A group gathers the calls of all its handles that arrive together into one
// launch (one wave per call): writers copy "history ‖ slice" into the open pinned staging
// buffer in parallel, the group thread seals it, ships it (H2D, kernel, D2H) while the
// writers fill the other buffer, and hands every writer its answer.
#ifndef KCDC_GROUP_ZC
#define KCDC_GROUP_ZC 1  // the scan reads the pinned staging in place (mapped), answers land in host memory
#endif
struct kcdc_group {
    const Algo* algo = nullptr;
    int device = 0;
    hipStream_t stream = nullptr;
    uint32_t max_batch = 0;
    std::chrono::microseconds wait{0};
    struct Buf {
        uint8_t* h = nullptr;  // pinned staging
        uint8_t* d = nullptr;  // its device copy, or (KCDC_GROUP_ZC) its device mapping
        uint8_t* scratch = nullptr;  // (KCDC_GROUP_ZC) device scratch the scan copies the staging into
        ScanReq* h_req = nullptr;
        ScanReq* d_req = nullptr;
        int64_t* h_out = nullptr;
        int64_t* d_out = nullptr;
        std::vector<int64_t*> result;  // each request's answer slot (the writer's stack)
        size_t used = 0;
        uint32_t n = 0, writing = 0;
        uint64_t seq = 0;
    };
    static constexpr size_t kCap = size_t(32) << 20;  // staging bytes per buffer
    Buf buf[2];
    int open = 0;
    uint64_t seq_next = 1, completed = 0;
    uint32_t live = 0;  // open handles: a launch is sealed at once when every one of them waits
    bool closing = false;  // kcdc_group_free was called with handles still open
    int error = 0;
    std::mutex mu;
    std::condition_variable cv_work, cv_done;
    bool stop = false;
    std::thread th;
};

namespace {

void group_release(kcdc_group* g) {
    DeviceGuard dg(g->device);
    for (auto& b : g->buf) {
        if (b.h) (void)hipHostFree(b.h);
        if (b.h_req) (void)hipHostFree(b.h_req);
        if (b.h_out) (void)hipHostFree(b.h_out);
        if (b.scratch) (void)hipFree(b.scratch);
        if (!KCDC_GROUP_ZC) {  // device copies (zero-copy: mappings of the host buffers)
            if (b.d) (void)hipFree(b.d);
            if (b.d_req) (void)hipFree(b.d_req);
            if (b.d_out) (void)hipFree(b.d_out);
        }
    }
    if (g->stream) (void)hipStreamDestroy(g->stream);
    delete g;
}

void group_loop(kcdc_group* g) {
    (void)hipSetDevice(g->device);
    std::unique_lock<std::mutex> lk(g->mu);
    for (;;) {
        g->cv_work.wait(lk, [&] { return g->stop || g->buf[g->open].n > 0; });
        if (g->stop && g->buf[g->open].n == 0) return;
        // let the writers that are arriving join this launch
        const auto deadline = std::chrono::steady_clock::now() + g->wait;
        g->cv_work.wait_until(lk, deadline, [&] {
            const uint32_t n = g->buf[g->open].n;
            return g->stop || n >= g->max_batch || n >= g->live;
        });
        kcdc_group::Buf& B = g->buf[g->open];
        g->open ^= 1;  // later writers fill the other buffer (idle: launches complete in order)
        g->buf[g->open].seq = g->seq_next++;
        g->cv_work.wait(lk, [&] { return B.writing == 0; });
        const uint32_t n = B.n;
        const size_t used = B.used;
        lk.unlock();
        int rc = KCDC_OK;
        hipError_t e = hipSuccess;
        if (KCDC_GROUP_ZC) {  // the kernel reads the staging and writes the answers over PCIe
            rc = launch_scan_first_batch(*g->algo, B.d, B.d_req, n, B.d_out, g->device, g->stream, B.scratch);
        } else {
            e = hipMemcpyAsync(B.d, B.h, used, hipMemcpyHostToDevice, g->stream);
            if (e == hipSuccess)
                e = hipMemcpyAsync(B.d_req, B.h_req, n * sizeof(ScanReq), hipMemcpyHostToDevice, g->stream);
            if (e == hipSuccess) {
                rc = launch_scan_first_batch(*g->algo, B.d, B.d_req, n, B.d_out, g->device, g->stream);
                if (rc == KCDC_OK)
                    e = hipMemcpyAsync(B.h_out, B.d_out, n * sizeof(int64_t), hipMemcpyDeviceToHost, g->stream);
            }
        }
        if (e == hipSuccess && rc == KCDC_OK) e = hipStreamSynchronize(g->stream);
        if (e != hipSuccess && rc == KCDC_OK) rc = KCDC_EIO;
        lk.lock();
        for (uint32_t k = 0; k < n; k++) *B.result[k] = rc == KCDC_OK ? B.h_out[k] : rc;
        B.n = 0;
        B.used = 0;
        g->completed = B.seq;
        g->cv_done.notify_all();
        g->cv_work.notify_all();  // writers waiting for room
    }
}

void group_shutdown(kcdc_group* g) {
    {
        std::lock_guard<std::mutex> lk(g->mu);
        g->stop = true;
    }
    g->cv_work.notify_all();
    if (g->th.joinable()) g->th.join();
    group_release(g);
}

void group_handle_closed(kcdc_group* g) {
    bool last = false;
    {
        std::lock_guard<std::mutex> lk(g->mu);
        g->live--;
        last = g->closing && g->live == 0;
        // Notify while holding the mutex: once it is released, the thread that shuts the
        // group down (the last closer, or kcdc_group_free seeing live == 0) may delete g.
        g->cv_work.notify_all();  // a pending launch may now hold every live handle
    }
    if (last) group_shutdown(g);  // kcdc_group_free came first: the last handle frees the group
}

int64_t group_first_candidate(kcdc_splitter* s, const uint8_t* b, size_t n) {
    kcdc_group* g = s->group;
    const size_t total = kWindow + n;
    const size_t need = (total + 255) & ~size_t(255);
    if (need > kcdc_group::kCap) return KCDC_EOVERFLOW;
    int64_t result = KCDC_EIO;
    std::unique_lock<std::mutex> lk(g->mu);
    g->cv_work.wait(lk, [&] {
        const kcdc_group::Buf& B = g->buf[g->open];
        return B.n < g->max_batch && B.used + need <= kcdc_group::kCap;
    });
    kcdc_group::Buf& B = g->buf[g->open];
    const uint32_t slot = B.n++;
    const size_t off = B.used;
    B.used += need;
    B.writing++;
    B.result[slot] = &result;
    const uint64_t seq = B.seq;
    lk.unlock();
    std::memcpy(B.h + off, s->hist, kWindow);  // staged by the writer's own thread
    std::memcpy(B.h + off + kWindow, b, n);
    B.h_req[slot] = ScanReq{off, static_cast<int64_t>(total), kWindow, static_cast<int64_t>(total) - 1};
    lk.lock();
    B.writing--;
    g->cv_work.notify_all();
    g->cv_done.wait(lk, [&] { return g->completed >= seq; });
    lk.unlock();
    if (result < -1) return set_error(static_cast<int>(result), "grouped scan failed");
    return result < 0 ? -1 : result - kWindow;
}

}  // namespace

extern "C" kcdc_group* kcdc_group_new(const char* name, int device, uint32_t max_batch, uint32_t max_wait_us) {
    const Algo* a = find_algo(name);
    if (!a) {
        set_error(KCDC_ENOENT, std::string("unknown splitter: ") + (name ? name : "(null)"));
        return nullptr;
    }
    if (a->kind == kFixed) {
        set_error(KCDC_EINVAL, "FIXED splitters read no data: use kcdc_splitter_new");
        return nullptr;
    }
    if (check_device(device) != KCDC_OK) return nullptr;
    DeviceGuard dg(device);
    int err = 0;
    if (!device_tables(device, &err)) return nullptr;
    kcdc_group* g = new kcdc_group();
    g->algo = a;
    g->device = device;
    g->max_batch = std::max<uint32_t>(1, std::min<uint32_t>(max_batch ? max_batch : 256, 4096));
    g->wait = std::chrono::microseconds(max_wait_us);
    bool ok = hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking) == hipSuccess;
    const unsigned hflags = KCDC_GROUP_ZC ? hipHostMallocMapped : hipHostMallocDefault;
    for (auto& b : g->buf) {
        ok = ok && hipHostMalloc(&b.h, kcdc_group::kCap, hflags) == hipSuccess &&
             hipHostMalloc(&b.h_req, g->max_batch * sizeof(ScanReq), hflags) == hipSuccess &&
             hipHostMalloc(&b.h_out, g->max_batch * sizeof(int64_t), hflags) == hipSuccess;
        if (ok && KCDC_GROUP_ZC) {
            void *pd = nullptr, *pr = nullptr, *po = nullptr;
            ok = hipHostGetDevicePointer(&pd, b.h, 0) == hipSuccess &&
                 hipHostGetDevicePointer(&pr, b.h_req, 0) == hipSuccess &&
                 hipHostGetDevicePointer(&po, b.h_out, 0) == hipSuccess;
            b.d = static_cast<uint8_t*>(pd);
            b.d_req = static_cast<ScanReq*>(pr);
            b.d_out = static_cast<int64_t*>(po);
            ok = ok && hipMalloc(&b.scratch, kcdc_group::kCap) == hipSuccess;
        } else if (ok) {
            ok = hipMalloc(&b.d, kcdc_group::kCap) == hipSuccess &&
                 hipMalloc(&b.d_req, g->max_batch * sizeof(ScanReq)) == hipSuccess &&
                 hipMalloc(&b.d_out, g->max_batch * sizeof(int64_t)) == hipSuccess;
        }
        if (ok) b.result.resize(g->max_batch);
    }
    if (!ok) {
        set_error(KCDC_ENOMEM, "failed to allocate splitter group resources");
        group_release(g);
        return nullptr;
    }
    g->buf[0].seq = g->seq_next++;
    g->th = std::thread(group_loop, g);
    return g;
}

extern "C" kcdc_splitter* kcdc_group_splitter(kcdc_group* g) {
    if (!g) {
        set_error(KCDC_EINVAL, "null group");
        return nullptr;
    }
    {
        std::lock_guard<std::mutex> lk(g->mu);
        if (g->closing) {  // kcdc_group_free was called: no new handles (kcdc.h)
            set_error(KCDC_EINVAL, "splitter group is being freed");
            return nullptr;
        }
    }
    DeviceGuard dg(g->device);
    kcdc_splitter* s = new kcdc_splitter();
    s->algo = g->algo;
    s->device = g->device;
    if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess ||
        alloc_out(s) != hipSuccess) {
        set_error(KCDC_EIO, "failed to allocate splitter device resources");
        destroy(s);
        return nullptr;
    }
    std::lock_guard<std::mutex> lk(g->mu);
    if (g->closing) {  // freed while the handle's resources were allocated
        set_error(KCDC_EINVAL, "splitter group is being freed");
        destroy(s);
        return nullptr;
    }
    s->group = g;
    g->live++;
    return s;
}

extern "C" void kcdc_group_free(kcdc_group* g) {
    if (!g) return;
    {
        std::lock_guard<std::mutex> lk(g->mu);
        if (g->live > 0) {  // handles still open: the last kcdc_splitter_close frees the group
            g->closing = true;
            return;
        }
    }
    group_shutdown(g);
}

// ==================================================================== batch
extern "C" int kcdc_split_batch_device(const char* name, const uint8_t* const* d_ptrs, const uint64_t* d_lens,
                                       uint32_t nstreams, uint64_t* d_cuts, uint64_t cuts_cap,
                                       const uint64_t* d_cut_base, uint64_t* d_counts, void* stream) {
    const Algo* a = find_algo(name);
    if (!a) return set_error(KCDC_ENOENT, std::string("unknown splitter: ") + (name ? name : "(null)"));
    if (nstreams == 0) return KCDC_OK;
    if (!d_ptrs || !d_lens || !d_cuts || !d_cut_base || !d_counts) return set_error(KCDC_EINVAL, "null argument");
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev), "hipGetDevice");
    int rc = check_device(dev);
    if (rc) return rc;
    SplitArgs s{d_ptrs, d_lens, nstreams, d_cuts, cuts_cap, d_cut_base, d_counts};
    return launch_split_batch(*a, s, dev, stream);
}

namespace {
// One slot of the host batch path: a device arena for a group's bytes, its cut lists, and
// pinned host copies of the answers (so the D2H never blocks the host thread).
struct HostSlot {
    uint8_t* d_data = nullptr;
    size_t d_data_cap = 0;
    void* d_meta = nullptr;
    size_t d_meta_cap = 0;
    uint64_t* h_meta = nullptr;  // pinned: counts then cuts of the group
    size_t h_meta_cap = 0;
    hipStream_t stream = nullptr;
    bool busy = false;
    uint32_t i0 = 0, i1 = 0;
    uint64_t gcap = 0;
};
struct HostCtx {
    std::mutex mu;
    HostSlot slot[2];
};
HostCtx g_host[64];

int grow(void** p, size_t* cap, size_t need) {
    if (need <= *cap) return KCDC_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    HIP_TRY(hipMalloc(p, need), "hipMalloc");
    *cap = need;
    return KCDC_OK;
}
int grow_pinned(uint64_t** p, size_t* cap, size_t need) {
    if (need <= *cap) return KCDC_OK;
    if (*p) (void)hipHostFree(*p);
    *p = nullptr;
    *cap = 0;
    HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(p), need, hipHostMallocDefault), "hipHostMalloc");
    *cap = need;
    return KCDC_OK;
}
// Wait for a slot's group and hand its answers to the caller's arrays.
int host_slot_finish(HostSlot& S, uint32_t nstreams, uint64_t* cuts, uint64_t cuts_cap, const uint64_t* cut_base,
                     uint64_t* counts) {
    if (!S.busy) return KCDC_OK;
    S.busy = false;
    HIP_TRY(hipStreamSynchronize(S.stream), "sync");
    const uint32_t ng = S.i1 - S.i0;
    std::memcpy(counts + S.i0, S.h_meta, ng * sizeof(uint64_t));
    if (S.gcap) std::memcpy(cuts + cut_base[S.i0], S.h_meta + ng, S.gcap * sizeof(uint64_t));
    for (uint32_t k = S.i0; k < S.i1; k++) {
        if (counts[k] == KCDC_COUNT_FAILED) return set_error(KCDC_EIO, "batch launch failed on the device");
        const uint64_t capk = (k + 1 < nstreams ? cut_base[k + 1] : cuts_cap) - cut_base[k];
        if (counts[k] > capk) return set_error(KCDC_EOVERFLOW, "cut capacity too small for a stream");
    }
    return KCDC_OK;
}
}  // namespace

// Host buffers in, cut lists out (snapshot/upload/upload.go:393-435 feeds the splitter from
// files in host memory).  Streams go in groups of at most kArena bytes through two slots on
// two HIP streams: while group k splits and its answers come back on one stream, group k+1's
// bytes go up on the other, so the PCIe H2D copy -- the bound of this path -- never waits for
// the GPU (the split of a 256 MiB group takes ~25 us against ~5 ms of transfer).
extern "C" int kcdc_split_batch_host(const char* name, const uint8_t* const* h_ptrs, const uint64_t* lens,
                                     uint32_t nstreams, uint64_t* cuts, uint64_t cuts_cap, const uint64_t* cut_base,
                                     uint64_t* counts, int device) {
    const Algo* a = find_algo(name);
    if (!a) return set_error(KCDC_ENOENT, std::string("unknown splitter: ") + (name ? name : "(null)"));
    if (nstreams == 0) return KCDC_OK;
    if (!h_ptrs || !lens || !cuts || !cut_base || !counts) return set_error(KCDC_EINVAL, "null argument");
    int rc = check_device(device);
    if (rc) return rc;
    DeviceGuard g(device);
    HostCtx& C = g_host[device];
    std::lock_guard<std::mutex> lk(C.mu);
    for (HostSlot& S : C.slot)
        if (!S.stream) HIP_TRY(hipStreamCreateWithFlags(&S.stream, hipStreamNonBlocking), "hipStreamCreate");
    // Groups of streams whose bytes fit one arena (a larger stream gets an arena of its own size).
    const size_t kArena = size_t(256) << 20;
    uint32_t i0 = 0, k = 0;
    while (i0 < nstreams) {
        uint32_t i1 = i0;
        size_t bytes = 0;
        while (i1 < nstreams) {
            const size_t sz = (lens[i1] + 255) & ~size_t(255);
            if (i1 > i0 && bytes + sz > kArena) break;
            bytes += sz;
            i1++;
        }
        HostSlot& S = C.slot[k++ & 1];
        rc = host_slot_finish(S, nstreams, cuts, cuts_cap, cut_base, counts);  // the group before last
        if (rc) break;
        const uint32_t ng = i1 - i0;
        const uint64_t gcap = (i1 < nstreams ? cut_base[i1] : cuts_cap) - cut_base[i0];
        rc = grow(reinterpret_cast<void**>(&S.d_data), &S.d_data_cap, std::max<size_t>(bytes, 256));
        if (!rc) rc = grow(&S.d_meta, &S.d_meta_cap, (ng + gcap) * sizeof(uint64_t) + 64);
        if (!rc) rc = grow_pinned(&S.h_meta, &S.h_meta_cap, (ng + gcap) * sizeof(uint64_t) + 64);
        if (rc) break;
        std::vector<const uint8_t*> dptr(ng);
        std::vector<uint64_t> base(ng);
        // Runs of streams that are adjacent in host memory go up as ONE copy (each pageable
        // copy call costs ~15 us of runtime staging: 1024 x 4 MiB copies lost 15% of the link);
        // inside a run the device keeps the host layout, each run starts 256-byte aligned.
        size_t off = 0;
        for (uint32_t j = 0; j < ng;) {
            uint32_t e = j + 1;
            size_t run = lens[i0 + j];
            while (e < ng && h_ptrs[i0 + e] == h_ptrs[i0 + e - 1] + lens[i0 + e - 1]) run += lens[i0 + e++];
            for (uint32_t q = j; q < e; q++) {
                dptr[q] = S.d_data + off + (h_ptrs[i0 + q] - h_ptrs[i0 + j]);
                base[q] = cut_base[i0 + q] - cut_base[i0];
            }
            if (run) {
                const hipError_t err = hipMemcpyAsync(S.d_data + off, h_ptrs[i0 + j], run, hipMemcpyHostToDevice, S.stream);
                if (err != hipSuccess) {
                    rc = set_error(KCDC_EIO, std::string("H2D stream: ") + hipGetErrorString(err));
                    break;
                }
            }
            off += (run + 255) & ~size_t(255);
            j = e;
        }
        if (rc) break;
        auto* d_cnt = static_cast<uint64_t*>(S.d_meta);
        auto* d_cuts = d_cnt + ng;
        // each stream through the batch kernel or, if it would be the batch's tail, the long path
        rc = kcdc_split_files_device(name, dptr.data(), lens + i0, ng, d_cuts, gcap, base.data(), d_cnt, S.stream);
        if (rc) break;
        const hipError_t e = hipMemcpyAsync(S.h_meta, S.d_meta, (ng + gcap) * sizeof(uint64_t), hipMemcpyDeviceToHost,
                                            S.stream);
        if (e != hipSuccess) {
            rc = set_error(KCDC_EIO, std::string("D2H: ") + hipGetErrorString(e));
            break;
        }
        S.busy = true;
        S.i0 = i0;
        S.i1 = i1;
        S.gcap = gcap;
        i0 = i1;
    }
    for (HostSlot& S : C.slot) {  // drain both slots, also after an error (no work left in flight)
        const int r2 = host_slot_finish(S, nstreams, cuts, cuts_cap, cut_base, counts);
        if (!rc) rc = r2;
    }
    return rc;
}

// Longest processing time first: streams by bytes, largest first (ties: lower index), each to
// the least-loaded of `ndev` devices (ties: lower index).  dev_of[i] = position of stream i's
// device.  Host arithmetic (kopia_amd/dist.py lpt_plan is the same rule).
extern "C" int kcdc_lpt_assign(const uint64_t* lens, uint32_t n, uint32_t ndev, uint32_t* dev_of) {
    if (n == 0) return KCDC_OK;
    if (!lens || !dev_of || ndev == 0) return set_error(KCDC_EINVAL, "null argument or no devices");
    std::vector<uint32_t> order(n);
    for (uint32_t i = 0; i < n; i++) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) { return lens[x] > lens[y]; });
    std::vector<uint64_t> load(ndev, 0);
    for (uint32_t i : order) {
        uint32_t d = 0;
        for (uint32_t k = 1; k < ndev; k++)
            if (load[k] < load[d]) d = k;
        dev_of[i] = d;
        load[d] += lens[i];
    }
    return KCDC_OK;
}

// kcdc_split_batch_host over a device set: the streams are spread by bytes (kcdc_lpt_assign) and
// every device runs the double-buffered host path on its share from a thread of its own; the
// answers land in the caller's arrays as for one device.  Files in host memory in, cut lists out,
// for a node's GPUs (no collectives, each device independent).
extern "C" int kcdc_split_batch_host_devices(const char* name, const int* devices, int ndev, const uint8_t* const* h_ptrs,
                                             const uint64_t* lens, uint32_t nstreams, uint64_t* cuts, uint64_t cuts_cap,
                                             const uint64_t* cut_base, uint64_t* counts) {
    const Algo* a = find_algo(name);
    if (!a) return set_error(KCDC_ENOENT, std::string("unknown splitter: ") + (name ? name : "(null)"));
    if (nstreams == 0) return KCDC_OK;
    if (!h_ptrs || !lens || !cuts || !cut_base || !counts) return set_error(KCDC_EINVAL, "null argument");
    std::vector<int> list;
    if (!devices || ndev <= 0) {
        const int nd = kcdc_device_count();
        if (nd <= 0) return set_error(KCDC_ENODEV, "no HIP device");
        for (int d = 0; d < nd; d++) list.push_back(d);
    } else {
        list.assign(devices, devices + ndev);
    }
    for (int d : list) {
        const int rc = check_device(d);
        if (rc) return rc;
    }
    for (uint32_t i = 0; i < nstreams; i++)
        if (cut_base[i] > cuts_cap || (i + 1 < nstreams && cut_base[i + 1] < cut_base[i]))
            return set_error(KCDC_EINVAL, "cut_base must be non-decreasing and within cuts_cap");
    const uint32_t nd = static_cast<uint32_t>(list.size());
    std::vector<uint32_t> dev_of(nstreams);
    (void)kcdc_lpt_assign(lens, nstreams, nd, dev_of.data());
    struct Share {
        std::vector<uint32_t> idx;
        std::vector<const uint8_t*> ptrs;
        std::vector<uint64_t> lens, base, counts, cuts;
        uint64_t cap = 0;
        int rc = KCDC_OK;
        std::string err;
    };
    std::vector<Share> sh(nd);
    for (uint32_t i = 0; i < nstreams; i++) {
        Share& S = sh[dev_of[i]];
        const uint64_t capi = (i + 1 < nstreams ? cut_base[i + 1] : cuts_cap) - cut_base[i];
        S.idx.push_back(i);
        S.ptrs.push_back(h_ptrs[i]);
        S.lens.push_back(lens[i]);
        S.base.push_back(S.cap);
        S.cap += capi;
    }
    std::vector<std::thread> th;
    for (uint32_t k = 0; k < nd; k++) {
        if (sh[k].idx.empty()) continue;
        th.emplace_back([&, k] {
            Share& S = sh[k];
            S.counts.assign(S.idx.size(), 0);
            S.cuts.assign(std::max<uint64_t>(S.cap, 1), 0);
            S.rc = kcdc_split_batch_host(name, S.ptrs.data(), S.lens.data(), static_cast<uint32_t>(S.idx.size()),
                                         S.cuts.data(), S.cap, S.base.data(), S.counts.data(), list[k]);
            if (S.rc) S.err = kcdc_last_error();
        });
    }
    for (auto& t : th) t.join();
    for (uint32_t k = 0; k < nd; k++)
        if (sh[k].rc) return set_error(sh[k].rc, "device " + std::to_string(list[k]) + ": " + sh[k].err);
    for (uint32_t k = 0; k < nd; k++) {
        const Share& S = sh[k];
        for (size_t j = 0; j < S.idx.size(); j++) {
            const uint32_t i = S.idx[j];
            counts[i] = S.counts[j];
            std::memcpy(cuts + cut_base[i], S.cuts.data() + S.base[j], S.counts[j] * sizeof(uint64_t));
        }
    }
    return KCDC_OK;
}

// ================================================================ long stream
extern "C" size_t kcdc_long_workspace_bytes(const char* name, uint64_t len) {
    const Algo* a = find_algo(name);
    return a ? long_workspace_bytes(*a, len) : 0;
}

extern "C" int kcdc_split_long_device(const char* name, const uint8_t* d_data, uint64_t len, uint64_t* d_cuts,
                                      uint64_t cuts_cap, uint64_t* d_count, void* ws, size_t ws_bytes, void* stream) {
    const Algo* a = find_algo(name);
    if (!a) return set_error(KCDC_ENOENT, std::string("unknown splitter: ") + (name ? name : "(null)"));
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev), "hipGetDevice");
    int rc = check_device(dev);
    if (rc) return rc;
    return launch_split_long(*a, d_data, len, d_cuts, cuts_cap, d_count, ws, ws_bytes, dev, stream);
}

// ================================================================ mixed sizes
namespace {
// Single-wave scan rate of the batch kernel and its whole-GPU rate (bytes/s, MI355X, round-1
// measurements): a stream whose lone-wave time exceeds the batch's aggregate time would be the
// batch's tail, so it goes to the long (intra-stream parallel) path instead.
constexpr double kWaveRate = 6e9, kBatchRate = 1.2e13;
constexpr uint64_t kLongMin = uint64_t(1) << 20;
}  // namespace

extern "C" int kcdc_split_files_device(const char* name, const uint8_t* const* h_dptrs, const uint64_t* h_lens,
                                       uint32_t n, uint64_t* d_cuts, uint64_t cuts_cap, const uint64_t* h_cut_base,
                                       uint64_t* d_counts, void* stream) {
    const Algo* a = find_algo(name);
    if (!a) return set_error(KCDC_ENOENT, std::string("unknown splitter: ") + (name ? name : "(null)"));
    if (n == 0) return KCDC_OK;
    if (!h_dptrs || !h_lens || !d_cuts || !h_cut_base || !d_counts) return set_error(KCDC_EINVAL, "null argument");
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev), "hipGetDevice");
    int rc = check_device(dev);
    if (rc) return rc;
    hipStream_t st = static_cast<hipStream_t>(stream);
    for (uint32_t i = 0; i < n; i++)
        if (h_cut_base[i] > cuts_cap || (i + 1 < n && h_cut_base[i + 1] < h_cut_base[i]))
            return set_error(KCDC_EINVAL, "cut_base must be non-decreasing and within cuts_cap");
    // Route: largest streams first to the long path while a lone wave on one would outlast
    // the rest of the batch (FIXED reads no data: always the batch entry point).
    std::vector<uint32_t> order(n);
    for (uint32_t i = 0; i < n; i++) order[i] = i;
    std::sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) { return h_lens[x] > h_lens[y]; });
    double rest = 0;
    for (uint32_t i = 0; i < n; i++) rest += static_cast<double>(h_lens[i]);
    std::vector<char> is_long(n, 0);
    if (a->kind != kFixed)
        for (uint32_t k = 0; k < n; k++) {
            const uint32_t i = order[k];
            const double L = static_cast<double>(h_lens[i]);
            if (h_lens[i] < kLongMin || L / kWaveRate <= (rest - L) / kBatchRate) break;
            is_long[i] = 1;
            rest -= L;
        }
    std::vector<const uint8_t*> bp, lp;
    std::vector<uint64_t> bl, bb, ll, lcap;
    std::vector<uint64_t*> lcuts, lcnt;
    std::vector<uint32_t> bidx;
    for (uint32_t i = 0; i < n; i++) {
        if (is_long[i]) {
            lp.push_back(h_dptrs[i]);
            ll.push_back(h_lens[i]);
            lcap.push_back((i + 1 < n ? h_cut_base[i + 1] : cuts_cap) - h_cut_base[i]);
            lcuts.push_back(d_cuts + h_cut_base[i]);
            lcnt.push_back(d_counts + i);
        } else {
            bidx.push_back(i);
            bp.push_back(h_dptrs[i]);
            bl.push_back(h_lens[i]);
            bb.push_back(h_cut_base[i]);
        }
    }
    if (!bidx.empty()) {  // one batch launch over the small streams, each keeping its cut range
        // counts[] of the batch go to a scratch array and are scattered to d_counts
        const uint32_t nb = static_cast<uint32_t>(bidx.size());
        const size_t meta = nb * (sizeof(void*) + 4 * sizeof(uint64_t));
        char* m = nullptr;
        HIP_TRY(hipMallocAsync(reinterpret_cast<void**>(&m), meta, st), "hipMallocAsync meta");
        auto* d_ptrs = reinterpret_cast<const uint8_t**>(m);
        auto* d_lens = reinterpret_cast<uint64_t*>(m + nb * sizeof(void*));
        auto* d_base = d_lens + nb;
        auto* d_cnt = d_base + nb;
        auto* d_end = d_cnt + nb;
        // Each batch stream's cut range ends where the caller's range for it ends (cut_end),
        // not at the next batch stream's base: a stream that overflows its range never writes
        // into the ranges of long streams placed between batch streams.
        HIP_TRY(hipMemcpyAsync(d_ptrs, bp.data(), nb * sizeof(void*), hipMemcpyHostToDevice, st), "H2D meta");
        HIP_TRY(hipMemcpyAsync(d_lens, bl.data(), nb * sizeof(uint64_t), hipMemcpyHostToDevice, st), "H2D meta");
        HIP_TRY(hipMemcpyAsync(d_base, bb.data(), nb * sizeof(uint64_t), hipMemcpyHostToDevice, st), "H2D meta");
        std::vector<uint64_t> be(nb);
        for (uint32_t k = 0; k < nb; k++) be[k] = bidx[k] + 1 < n ? h_cut_base[bidx[k] + 1] : cuts_cap;
        HIP_TRY(hipMemcpyAsync(d_end, be.data(), nb * sizeof(uint64_t), hipMemcpyHostToDevice, st), "H2D meta");
        SplitArgs sa{d_ptrs, d_lens, nb, d_cuts, cuts_cap, d_base, d_cnt, d_end};
        rc = launch_split_batch(*a, sa, dev, stream);
        if (rc) {
            (void)hipFreeAsync(m, st);
            return rc;
        }
        for (uint32_t k = 0; k < nb; k++)  // runs of consecutive indices copy as one
            if (k == 0 || bidx[k] != bidx[k - 1] + 1) {
                uint32_t e = k + 1;
                while (e < nb && bidx[e] == bidx[e - 1] + 1) e++;
                HIP_TRY(hipMemcpyAsync(d_counts + bidx[k], d_cnt + k, (e - k) * sizeof(uint64_t),
                                       hipMemcpyDeviceToDevice, st),
                        "scatter counts");
            }
        HIP_TRY(hipFreeAsync(m, st), "hipFreeAsync meta");
    }
    if (!lp.empty()) {  // every long stream in one long-path launch
        const uint32_t m = static_cast<uint32_t>(lp.size());
        const size_t wsb = long_workspace_bytes_multi(*a, ll.data(), m);
        void* ws = nullptr;
        HIP_TRY(hipMallocAsync(&ws, wsb, st), "hipMallocAsync long workspace");
        rc = launch_split_long_multi(*a, m, lp.data(), ll.data(), lcuts.data(), lcap.data(), lcnt.data(), ws, wsb,
                                     dev, stream);
        (void)hipFreeAsync(ws, st);
    }
    return rc;
}

// =================================================================== data
extern "C" int kcdc_fill_prng(uint8_t* d_data, uint64_t stride, uint64_t stream_len, uint32_t nstreams, uint64_t seed,
                              uint64_t first_sid, void* stream) {
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev), "hipGetDevice");
    int rc = check_device(dev);
    if (rc) return rc;
    return launch_fill_prng(d_data, stride, stream_len, nstreams, seed, first_sid, stream);
}

extern "C" int kcdc_gorand_read(int64_t seed, uint8_t* out, uint64_t n) {
    if (n && !out) return set_error(KCDC_EINVAL, "null buffer");
    gorand_read(seed, out, n);
    return KCDC_OK;
}
